// hg_gemm.hip — LDS-staged f32 GEMM of the policy MLPs on the f32 matrix cores (gfx950,
// v_mfma_f32_32x32x2_f32: exact f32 products, f32 accumulation) with the layer's elementwise work
// in the epilogue, so no separate ELU / ELU-backward pass touches the [rows, width] tensors.
//
// Two products of a hidden layer (actor_critic.py:36-149: nn.Linear followed by nn.ELU):
//   forward   y  = elu(x W^T + b)            x [M, K] (row stride lda), W [N, K] row-major
//   input grad gh = (g W) * elu'(y_prev)     g [M, K] (lda), W [K, N] row-major, y_prev [M, N]
// The second is the dX GEMM of layer i fused with the ELU backward of layer i-1 (whose output
// y_prev is layer i's input; elu'(h) = y + 1 for y <= 0), plus the per-block column partial sums of
// gh — layer i-1's bias gradient, reduced later by the batched column-sum launch (hg_colsum_jobs).
//
// Mapping.  Block = WGM x WGN waves over a BM x BN output tile (each wave a (32 TM) x (32 TN) tile
// of 32x32 MFMA accumulators); the reduction runs in BK-wide chunks staged global -> registers ->
// LDS (double-buffered LDS, one barrier per chunk; the next chunk's global loads are issued before
// the current chunk's MFMAs).  Inside a chunk, k = 8q + 4h + s: lane (i, h) of a wave reads the
// float4 (s = 0..3) of its row i for k group q, which feeds four MFMAs (step s takes k = 8q + 4h +
// s from lane half h: the 32x32x2 maps are A[i][k = h], B[k = h][j = i]; a permutation of the k
// order inside the chunk, the same dot product).  LDS image (lds_off): layout 0 puts (q, r) rows
// of 8 floats one after another (lane reads at 32 i + 16 h bytes); layout 1 makes the 64 lanes'
// float4 reads one contiguous 1 KB run, with a 32-byte pad per q block that spreads the staging
// writes of one row's q groups over different banks.
// k-contiguous operands (x, g, W of the forward) are staged as 32-byte row segments (two 16-byte
// loads per thread, BK / 8 threads per row segment); the n-contiguous W of the input-gradient
// product as 4 scalar loads per thread (64 lanes = 64 consecutive n: 256 contiguous bytes per load
// instruction) written as one float4 of 4 consecutive k.
// Tails: rows / columns past the end read a clamped valid row and are not stored; k past the end
// reads 0 (only the last chunk takes the guarded path).  Blocks: XCD-aware order (consecutive
// logical tiles, i.e. one row band's column tiles, on one XCD's L2).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "hg_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));

struct GemmArgs {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  const float* bias;  // forward: [N] or null
  const float* Y;     // input grad: y_prev [M, N] (ldY) for the ELU backward
  int64_t ldY;
  float* C;
  int64_t ldc;
  float* colpart;  // input grad: [tiles_m, N] column partial sums of C, or null
  int64_t M;
  int N, K;
  int tiles_n;
  int64_t tiles;
  // forward (mode 0) column split: columns >= nsplit (> 0, a multiple of every tile's BN) go to C2
  // (ldc2) at column - nsplit, so one GEMM writes two contiguous outputs (zero: no split)
  float* C2;
  int64_t ldc2;
  int nsplit;
  const float* bias2;  // the bias of the columns >= nsplit (bias2[c - nsplit])
};

template <int LAY>
__device__ __forceinline__ int lds_off(int q, int R, int r, int h) {
  if (LAY == 0) return (q * (R + 1) + r) * 8 + 4 * h;
  return q * (8 * R + 8) + ((r >> 5) * 2 + h) * 128 + 4 * (r & 31);
}
template <int LAY>
constexpr int lds_floats(int R, int BK) {
  return LAY == 0 ? (BK / 8) * (R + 1) * 8 : (BK / 8) * (8 * R + 8);
}

// k-contiguous operand (row r at P + r * ld): R rows x BK k of the chunk at kc.  Item j: idx = tid
// + j NT, row = idx / QG, q = idx % QG (QG = BK / 8 threads per row segment).
template <int R, int BK, int NT>
constexpr int kc_items() { return (R * (BK / 8) + NT - 1) / NT; }
template <int R, int BK, int NT>
constexpr int nc_items() { return (R * (BK / 4) + NT - 1) / NT; }

template <int R, int BK, int NT, bool VEC, bool TAIL>
__device__ __forceinline__ void stage_kc_load(const float* __restrict__ P, int64_t ld, int64_t r0, int64_t rmax, int kc,
                                              int K, int tid, float v[kc_items<R, BK, NT>()][8]) {
  constexpr int QG = BK / 8;
#pragma unroll
  for (int j = 0; j < kc_items<R, BK, NT>(); j++) {
    const int idx = tid + j * NT;
    if ((R * QG) % NT != 0 && idx >= R * QG) break;
    const int row = idx / QG, q = idx % QG;
    const int64_t r = min<int64_t>(r0 + row, rmax);
    const int k0 = kc + 8 * q;
    const float* p = P + r * ld + k0;
    if (!TAIL) {
      if (VEC) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        v[j][0] = a.x; v[j][1] = a.y; v[j][2] = a.z; v[j][3] = a.w;
        v[j][4] = b.x; v[j][5] = b.y; v[j][6] = b.z; v[j][7] = b.w;
      } else {
        const f32x4u a = *reinterpret_cast<const f32x4u*>(p);
        const f32x4u b = *reinterpret_cast<const f32x4u*>(p + 4);
#pragma unroll
        for (int s = 0; s < 4; s++) {
          v[j][s] = a[s];
          v[j][4 + s] = b[s];
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; s++) v[j][s] = (k0 + s < K) ? p[s] : 0.f;
    }
  }
}

template <int R, int BK, int NT, int LAY>
__device__ __forceinline__ void stage_kc_store(float* __restrict__ S, int tid, const float v[kc_items<R, BK, NT>()][8]) {
  constexpr int QG = BK / 8;
#pragma unroll
  for (int j = 0; j < kc_items<R, BK, NT>(); j++) {
    const int idx = tid + j * NT;
    if ((R * QG) % NT != 0 && idx >= R * QG) break;
    const int row = idx / QG, q = idx % QG;
    *reinterpret_cast<float4*>(S + lds_off<LAY>(q, R, row, 0)) = make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
    *reinterpret_cast<float4*>(S + lds_off<LAY>(q, R, row, 1)) = make_float4(v[j][4], v[j][5], v[j][6], v[j][7]);
  }
}

// n-contiguous operand (element (n, k) at P[k * ld + n]): R columns x BK k.  Item j: idx = tid +
// j NT, n = idx % R, k4 = idx / R (4 consecutive k).
template <int R, int BK, int NT, bool TAIL>
__device__ __forceinline__ void stage_nc_load(const float* __restrict__ P, int64_t ld, int n0, int nmax, int kc, int K,
                                              int tid, float v[nc_items<R, BK, NT>()][4]) {
#pragma unroll
  for (int j = 0; j < nc_items<R, BK, NT>(); j++) {
    const int idx = tid + j * NT;
    if ((R * (BK / 4)) % NT != 0 && idx >= R * (BK / 4)) break;
    const int n = min(n0 + idx % R, nmax);
    const int k = kc + 4 * (idx / R);
#pragma unroll
    for (int s = 0; s < 4; s++) v[j][s] = (!TAIL || k + s < K) ? P[(int64_t)(k + s) * ld + n] : 0.f;
  }
}

template <int R, int BK, int NT, int LAY>
__device__ __forceinline__ void stage_nc_store(float* __restrict__ S, int tid, const float v[nc_items<R, BK, NT>()][4]) {
#pragma unroll
  for (int j = 0; j < nc_items<R, BK, NT>(); j++) {
    const int idx = tid + j * NT;
    if ((R * (BK / 4)) % NT != 0 && idx >= R * (BK / 4)) break;
    const int n = idx % R, k4 = idx / R;
    *reinterpret_cast<float4*>(S + lds_off<LAY>(k4 >> 1, R, n, k4 & 1)) =
        make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
  }
}

template <int BM, int BN, int BK, int LAY, int TM, int TN>
__device__ __forceinline__ void mma_chunk(const float* __restrict__ As, const float* __restrict__ Bs, int wm0, int wn0,
                                          int i, int h, f32x16 acc[TM][TN]) {
#pragma unroll
  for (int q = 0; q < BK / 8; q++) {
    float4 a[TM], b[TN];
#pragma unroll
    for (int m = 0; m < TM; m++) a[m] = *reinterpret_cast<const float4*>(As + lds_off<LAY>(q, BM, wm0 + 32 * m + i, h));
#pragma unroll
    for (int n = 0; n < TN; n++) b[n] = *reinterpret_cast<const float4*>(Bs + lds_off<LAY>(q, BN, wn0 + 32 * n + i, h));
#pragma unroll
    for (int m = 0; m < TM; m++)
#pragma unroll
      for (int n = 0; n < TN; n++) {
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].x, b[n].x, acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].y, b[n].y, acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].z, b[n].z, acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].w, b[n].w, acc[m][n], 0, 0, 0);
      }
  }
}

// MODE 0: forward (B k-contiguous [N, K]; + bias, ELU if ELU).  MODE 1: input grad (B n-contiguous
// [K, N]; ELU backward from Y when ELU; column partials when colpart is non-null).
// Epilogues shared by the MFMA GEMMs.  acc register q of a 32x32 tile: row (q & 3) + 8 (q >> 2) +
// 4h, column i.  Round 5: every global load an epilogue needs is issued up front and
// unconditionally (clamped addresses) — the bias once per column, Y sixteen rows at a time — so no
// wait on a load lands between two stores.  Written as before (load inside the store guard), the
// compiler waited for each Y load right before its store (32-64 dependent HBM round trips per wave
// in the input-gradient kernels) and re-waited vmcnt(0) for the bias before every store of the
// forward (stores count on that counter too).  Values, stores and the column-sum order unchanged.
template <int TM, int TN, bool ELU, bool BIAS>
__device__ __forceinline__ void epi_forward(const f32x16 (&acc)[TM][TN], const GemmArgs& g, float* __restrict__ C,
                                            int64_t row0, int col0, int i, int h, int64_t ldc, int cshift,
                                            const float* __restrict__ bias) {
  const int64_t mmax = g.M - 1;
  const int nmax = g.N - 1;
#pragma unroll
  for (int n = 0; n < TN; n++) {
    const int cidx = col0 + 32 * n + i;
    float bc = 0.f;
    if (BIAS) bc = bias[min(cidx, nmax) - cshift];
    asm volatile("" : "+v"(bc));  // the bias load retires here, once
    if (cidx > nmax) continue;
#pragma unroll
    for (int m = 0; m < TM; m++) {
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int64_t r = row0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (r <= mmax) {
          float v = acc[m][n][q] + bc;
          if (ELU) v = v > 0.f ? v : expm1f(v);
          C[r * ldc + cidx - cshift] = v;
        }
      }
    }
  }
}

// input gradient: C = acc * elu'(Y) (ELU) and the wave's column sums of the stored values (0 past
// the edges), per column n in cs[n]
template <int TM, int TN, bool ELU>
__device__ __forceinline__ void epi_input_grad(const f32x16 (&acc)[TM][TN], const GemmArgs& g, int64_t row0, int col0,
                                               int i, int h, float (&cs)[TN]) {
  const int64_t mmax = g.M - 1;
  const int nmax = g.N - 1;
#pragma unroll
  for (int n = 0; n < TN; n++) {
    const int cidx = col0 + 32 * n + i;
    const int cc = min(cidx, nmax);
    cs[n] = 0.f;
#pragma unroll
    for (int m = 0; m < TM; m++) {
      float yv[16];
      if (ELU) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int64_t r = row0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
          yv[q] = g.Y[min(r, mmax) * g.ldY + cc];
        }
      }
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int64_t r = row0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
        float v = acc[m][n][q];
        if (r <= mmax && cidx <= nmax) {
          if (ELU) v = yv[q] > 0.f ? v : v * (yv[q] + 1.f);
          g.C[r * g.ldc + cidx] = v;
        } else {
          v = 0.f;
        }
        cs[n] += v;
      }
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int BK, int LAY, int PIPE, bool VEC, int MODE, bool ELU>
__global__ void __launch_bounds__(64 * WGM * WGN) k_gemm(GemmArgs g) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int TM = BM / WGM / 32, TN = BN / WGN / 32;
  constexpr int SA = lds_floats<LAY>(BM, BK), SB = lds_floats<LAY>(BN, BK);  // floats per stage buffer
  static_assert(TM >= 1 && TN >= 1 && BM == 32 * TM * WGM && BN == 32 * TN * WGN, "wave tiling");
  static_assert(2 * (SA + SB) >= WGM * BN, "epilogue reduction buffer fits the staging LDS");
  __shared__ __attribute__((aligned(16))) float lds[2 * (SA + SB)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const unsigned nb = gridDim.x;
  unsigned L = blockIdx.x;
  if ((nb & 7u) == 0) L = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
  if ((int64_t)L >= g.tiles) return;  // whole block exits before any barrier
  const int64_t tm_idx = (int64_t)L / g.tiles_n;
  const int64_t m0 = tm_idx * BM;
  const int n0 = (int)((int64_t)L % g.tiles_n) * BN;
  const int wm0 = (wave % WGM) * (32 * TM), wn0 = (wave / WGM) * (32 * TN);
  const int64_t mmax = g.M - 1;
  const int nmax = g.N - 1;
  const int K = g.K;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; m++)
#pragma unroll
    for (int n = 0; n < TN; n++) acc[m][n] = (f32x16)0.f;

  constexpr int IA = kc_items<BM, BK, NT>();
  constexpr int IBK = kc_items<BN, BK, NT>(), IBN = nc_items<BN, BK, NT>();
  float va[IA][8];
  float vbk[MODE == 0 ? IBK : 1][8];
  float vbn[MODE == 1 ? IBN : 1][4];

  const int kfull = K & ~(BK - 1);
  const int nchunks = (K + BK - 1) / BK;
#define HG_STAGE_LOAD(KC, TAILV)                                                                  \
  do {                                                                                            \
    stage_kc_load<BM, BK, NT, VEC, TAILV>(g.A, g.lda, m0, mmax, KC, K, tid, va);                 \
    if (MODE == 0) stage_kc_load<BN, BK, NT, VEC, TAILV>(g.B, g.ldb, n0, nmax, KC, K, tid, vbk); \
    else stage_nc_load<BN, BK, NT, TAILV>(g.B, g.ldb, n0, nmax, KC, K, tid, vbn);                \
  } while (0)
#define HG_STAGE_STORE(BUF)                                               \
  do {                                                                    \
    stage_kc_store<BM, BK, NT, LAY>(BUF, tid, va);                        \
    if (MODE == 0) stage_kc_store<BN, BK, NT, LAY>((BUF) + SA, tid, vbk); \
    else stage_nc_store<BN, BK, NT, LAY>((BUF) + SA, tid, vbn);           \
  } while (0)
  if (kfull > 0) HG_STAGE_LOAD(0, false);
  else HG_STAGE_LOAD(0, true);
  HG_STAGE_STORE(lds);
  if (PIPE == 0) {
    // loads of chunk c + 1 issued at the head of iteration c, stored after its MFMAs
    __syncthreads();
    for (int c = 0; c < nchunks; c++) {
      float* cur = lds + (c & 1) * (SA + SB);
      float* nxt = lds + ((c + 1) & 1) * (SA + SB);
      const int kn = (c + 1) * BK;
      const bool more = c + 1 < nchunks;
      if (more) {
        if (kn < kfull) HG_STAGE_LOAD(kn, false);
        else HG_STAGE_LOAD(kn, true);
      }
      mma_chunk<BM, BN, BK, LAY, TM, TN>(cur, cur + SA, wm0, wn0, i, h, acc);
      if (more) HG_STAGE_STORE(nxt);
      __syncthreads();
    }
  } else {
    // one iteration of slack: chunk c + 1 (loaded during iteration c - 1) is stored at the head of
    // iteration c, then chunk c + 2's loads are issued into the freed registers
    if (nchunks > 1) {
      if (BK < kfull) HG_STAGE_LOAD(BK, false);
      else HG_STAGE_LOAD(BK, true);
    }
    __syncthreads();
    for (int c = 0; c < nchunks; c++) {
      float* cur = lds + (c & 1) * (SA + SB);
      float* nxt = lds + ((c + 1) & 1) * (SA + SB);
      if (c + 1 < nchunks) HG_STAGE_STORE(nxt);
      const int kn = (c + 2) * BK;
      if (c + 2 < nchunks) {
        if (kn < kfull) HG_STAGE_LOAD(kn, false);
        else HG_STAGE_LOAD(kn, true);
      }
      mma_chunk<BM, BN, BK, LAY, TM, TN>(cur, cur + SA, wm0, wn0, i, h, acc);
      __syncthreads();
    }
  }
#undef HG_STAGE_LOAD
#undef HG_STAGE_STORE

  // epilogue (epi_forward / epi_input_grad)
  if (MODE == 0) {
    if (g.bias) epi_forward<TM, TN, ELU, true>(acc, g, g.C, m0 + wm0, n0 + wn0, i, h, g.ldc, 0, g.bias);
    else epi_forward<TM, TN, ELU, false>(acc, g, g.C, m0 + wm0, n0 + wn0, i, h, g.ldc, 0, g.bias);
  } else {
    float* red = lds;  // [WGM][BN] column partials of the waves along M (staging buffers are free)
    float cs[TN];
    epi_input_grad<TM, TN, ELU>(acc, g, m0 + wm0, n0 + wn0, i, h, cs);
#pragma unroll
    for (int n = 0; n < TN; n++) {
      const int cl = wn0 + 32 * n + i;
      cs[n] += __shfl_xor(cs[n], 32);
      if (h == 0) red[(wave % WGM) * BN + cl] = cs[n];
    }
    if (g.colpart) {
      __syncthreads();
      for (int c = tid; c < BN; c += NT) {
        if (n0 + c <= nmax) {
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < WGM; w++) s += red[w * BN + c];
          g.colpart[tm_idx * g.N + n0 + c] = s;
        }
      }
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int BK, int LAY, int PIPE = 0>
int launch(int mode, GemmArgs g, bool vec, bool elu, hipStream_t s) {
  g.tiles_n = (g.N + BN - 1) / BN;
  const int64_t tiles_m = (g.M + BM - 1) / BM;
  g.tiles = tiles_m * g.tiles_n;
  if (g.tiles > 0x7fffffff) return HG_ERR_ARG;
  const dim3 grid((unsigned)g.tiles), block(64 * WGM * WGN);
#define HG_G(V, MD, E) hipLaunchKernelGGL((k_gemm<BM, BN, WGM, WGN, BK, LAY, PIPE, V, MD, E>), grid, block, 0, s, g)
  if (mode == 0) {
    if (vec && elu) HG_G(true, 0, true);
    else if (vec) HG_G(true, 0, false);
    else if (elu) HG_G(false, 0, true);
    else HG_G(false, 0, false);
  } else {
    if (vec && elu) HG_G(true, 1, true);
    else if (vec) HG_G(true, 1, false);
    else if (elu) HG_G(false, 1, true);
    else HG_G(false, 1, false);
  }
#undef HG_G
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

// ---------------------------------------------------------------------------------------------
// f32 GEMM on the bf16 matrix cores (16x the f32 MFMA rate): every f32 operand is split exactly
// into three bf16 terms x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1):
// 24 significand bits; the rounding of x2 leaves ~2^-24 |x|, f32's own representation error), and
// the product keeps the six terms of total order <= 2, a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 +
// a2 b0 (the dropped a1 b2 + a2 b1 + a2 b2 are ~2^-24 |a b|), each bf16 x bf16 product exact in the
// f32 accumulator of v_mfma_f32_32x32x16_bf16, smallest terms first.  Measured error per element
// <= 3.4e-7 of sum_k |a_k b_k| (torch's f32 GEMM: 4.6e-7; tests/test_gpu_gemm.py bounds both at
// 1e-6).  The split runs once per element while the chunk is staged (global f32 -> registers ->
// three bf16 planes in LDS).
//   mode 0 forward     C = act(A B^T + bias)        A [M, K] k-contiguous, B [N, K] k-contiguous
//   mode 1 input grad  C = (A B) * elu'(Y) + colpart A [M, K] k-contiguous, B [K, N] n-contiguous
//   mode 2 weight grad C_s = sum_{k in slice s} A[k][m] B[k][n]   (A [K, M], B [K, N]: both
//          reduction-major; split-K slices of kslice rows write C + s * cstride, summed later in
//          fixed order by hg_colsum_jobs)
// Block BM x BN on WGM x WGN waves (each (32 TM) x (32 TN) of 32x32 accumulators), KG 16-deep k
// groups per staged chunk, double-buffered.  Plane image of an R-row operand tile: slot ((kg R /
// 32 + r / 32) 2 + h) 32 + r % 32 holds 8 bf16 (k = 16 kg + 8 h + 0..7): the 64 lanes' fragment
// reads are one contiguous 1 KB run.  k-contiguous operands are staged as two 16-byte loads per
// 8-k item; reduction-major ones as 8 scalar loads (64 lanes = 64 consecutive rows: 256 contiguous
// bytes per load instruction).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3x8(const float v[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const __bf16 a = (__bf16)v[j];
    const float r1 = v[j] - (float)a;
    const __bf16 b = (__bf16)r1;
    const float r2 = r1 - (float)b;
    h[j] = a;
    m[j] = b;
    l[j] = (__bf16)r2;
  }
}

__device__ __forceinline__ int x6_slot(int R, int kg, int r, int h) {
  return ((kg * (R >> 5) + (r >> 5)) * 2 + h) * 32 + (r & 31);
}

struct GemmX6Args {
  GemmArgs g;
  int64_t kslice;   // mode 2: reduction rows per split-K slice (multiple of 16)
  int64_t cstride;  // mode 2: elements between slices' outputs
  int slices;
};

// one operand's staging: R rows x (16 KG) k of the chunk at reduction index kc.  KC:
// k-contiguous rows (row r at P + r ld): items (r, 8-k piece), two 16-byte loads each;
// reduction-major (element (r, k) at P[k ld + r]): items (r, 8-k piece), eight scalar loads each
// (64 lanes = 64 consecutive r: 256 contiguous bytes per load instruction).  (Items of four r
// with 16-byte loads were measured 2-3x slower: a quarter of the threads carried the staging.)
template <int R, int KG, int NT, bool KC, bool VEC>
struct X6Stage {
  static constexpr int ITEMS = R * 2 * KG;
  static constexpr int IPT = (ITEMS + NT - 1) / NT;
  float v[IPT][8];
  __device__ __forceinline__ void item(int idx, int& r, int& piece) const {
    if (KC) { r = idx / (2 * KG); piece = idx % (2 * KG); }
    else { r = idx % R; piece = idx / R; }
  }
  // elements at or past kend read 0; rows past rmax read row rmax
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int64_t r0, int64_t rmax, int64_t kc,
                                       int64_t kend, bool tail, int tid) {
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int idx = tid + j * NT;
      if (ITEMS % NT != 0 && idx >= ITEMS) break;
      int r, piece;
      item(idx, r, piece);
      const int64_t rr = min<int64_t>(r0 + r, rmax);
      const int64_t k0 = kc + 8 * piece;
      if (KC) {
        const float* p = P + rr * ld + k0;
        if (!tail) {
          if (VEC) {
            const float4 x = *reinterpret_cast<const float4*>(p), y = *reinterpret_cast<const float4*>(p + 4);
            v[j][0] = x.x; v[j][1] = x.y; v[j][2] = x.z; v[j][3] = x.w;
            v[j][4] = y.x; v[j][5] = y.y; v[j][6] = y.z; v[j][7] = y.w;
          } else {
            const f32x4u x = *reinterpret_cast<const f32x4u*>(p), y = *reinterpret_cast<const f32x4u*>(p + 4);
#pragma unroll
            for (int q = 0; q < 4; q++) { v[j][q] = x[q]; v[j][4 + q] = y[q]; }
          }
        } else {
#pragma unroll
          for (int q = 0; q < 8; q++) v[j][q] = (k0 + q < kend) ? p[q] : 0.f;
        }
      } else {
        const float* p = P + k0 * ld + rr;
#pragma unroll
        for (int q = 0; q < 8; q++) v[j][q] = (!tail || k0 + q < kend) ? p[q * ld] : 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(bf16x8* __restrict__ plane0, int tid) const {
    constexpr int PS = R * 2 * KG;  // slots per plane
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int idx = tid + j * NT;
      if (ITEMS % NT != 0 && idx >= ITEMS) break;
      int r, piece;
      item(idx, r, piece);
      const int sl = x6_slot(R, piece >> 1, r, piece & 1);
      bf16x8 x0, x1, x2;
      split3x8(v[j], x0, x1, x2);
      plane0[sl] = x0;
      plane0[PS + sl] = x1;
      plane0[2 * PS + sl] = x2;
    }
  }
};

// reduction-major operand (element (r, k) at P[k ld + r], r contiguous) staged through an f32 LDS
// scratch: items (k row q, 4 consecutive r) read as 16-byte row segments (lanes along r, balanced
// over all threads), written transposed into scratch [R][16 KG + 1] (odd pitch: the lanes' 4-byte
// writes fall on distinct banks), then, after a barrier, every thread gathers one (r, 8-k piece)
// from the scratch, splits it and writes the three planes.
template <int R, int KG, int NT>
struct X6StageT {
  static constexpr int PITCH = 16 * KG + 1;
  static constexpr int ITEMS = 16 * KG * (R / 4);
  static constexpr int IPT = (ITEMS + NT - 1) / NT;
  static constexpr int PITEMS = R * 2 * KG;
  static constexpr int PIPT = (PITEMS + NT - 1) / NT;
  static constexpr int SCRATCH = R * PITCH;  // floats
  float v[IPT][4];
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int64_t r0, int64_t rmax, int64_t kc,
                                       int64_t kend, bool tail, int tid) {
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int idx = tid + j * NT;
      if (ITEMS % NT != 0 && idx >= ITEMS) break;
      const int g = idx % (R / 4), q = idx / (R / 4);
      const int64_t k = kc + q;
      const int64_t rr = r0 + 4 * g;
      const float* p = P + k * ld;
      const bool ok = !tail || k < kend;
      if (rr + 3 <= rmax) {
        f32x4u x = {0.f, 0.f, 0.f, 0.f};
        if (ok) x = *reinterpret_cast<const f32x4u*>(p + rr);
        v[j][0] = x[0]; v[j][1] = x[1]; v[j][2] = x[2]; v[j][3] = x[3];
      } else {
#pragma unroll
        for (int c = 0; c < 4; c++) v[j][c] = ok ? p[min<int64_t>(rr + c, rmax)] : 0.f;
      }
    }
  }
  __device__ __forceinline__ void to_scratch(float* __restrict__ sc, int tid) const {
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int idx = tid + j * NT;
      if (ITEMS % NT != 0 && idx >= ITEMS) break;
      const int g = idx % (R / 4), q = idx / (R / 4);
#pragma unroll
      for (int c = 0; c < 4; c++) sc[(4 * g + c) * PITCH + q] = v[j][c];
    }
  }
  __device__ __forceinline__ void to_planes(bf16x8* __restrict__ plane0, const float* __restrict__ sc, int tid) const {
    constexpr int PS = R * 2 * KG;
#pragma unroll
    for (int j = 0; j < PIPT; j++) {
      const int idx = tid + j * NT;
      if (PITEMS % NT != 0 && idx >= PITEMS) break;
      const int r = idx % R, piece = idx / R;
      float w[8];
#pragma unroll
      for (int q = 0; q < 8; q++) w[q] = sc[r * PITCH + 8 * piece + q];
      const int sl = x6_slot(R, piece >> 1, r, piece & 1);
      bf16x8 x0, x1, x2;
      split3x8(w, x0, x1, x2);
      plane0[sl] = x0;
      plane0[PS + sl] = x1;
      plane0[2 * PS + sl] = x2;
    }
  }
};

// the staging of one operand: k-contiguous (X6Stage, KC), reduction-major transposed through the
// LDS scratch (X6StageT), selected at compile time
template <int R, int KG, int NT, bool KC, bool VEC>
struct X6Op {
  X6Stage<R, KG, NT, true, VEC> kc;
  X6StageT<R, KG, NT> rt;
  static constexpr int SCRATCH = KC ? 0 : X6StageT<R, KG, NT>::SCRATCH;
  __device__ __forceinline__ void load(const float* P, int64_t ld, int64_t r0, int64_t rmax, int64_t kc0, int64_t kend,
                                       bool tail, int tid) {
    if (KC) kc.load(P, ld, r0, rmax, kc0, kend, tail, tid);
    else rt.load(P, ld, r0, rmax, kc0, kend, tail, tid);
  }
};

// IMG bit 0 (B) / bit 1 (A): the operand comes as a pre-split image (hg_gemm_x6_image_jobs; layout
// at k_x6_image_jobs): per 16-deep k chunk and plane, 32 rows form one contiguous 1 KB unit in
// exactly the LDS fragment order, so a block's BM (BN) rows of a chunk are copied by LDS-DMA
// (global_load_lds, 1 KB per wave instruction, lane-linear) with no register staging, split or LDS
// write pass.  The image's plane pitch (16-byte slots) rides in lda / ldb.
// APF (B from its image, A staged from k-contiguous rows): A's global loads run two chunks ahead
// in two register sets, so the activations' HBM latency has two chunks of MFMAs to hide behind
// (the B image comes from L2 by LDS-DMA one chunk ahead as before); same products, same bits
template <int BM, int BN, int WGM, int WGN, int KG, bool VEC, int MODE, bool ELU, int IMG = 0, bool APF = false>
__device__ __forceinline__ void gemm_x6_body(const GemmX6Args& xa) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int TM = BM / WGM / 32, TN = BN / WGN / 32;
  constexpr int PA = BM * 2 * KG, PB = BN * 2 * KG;  // 16-byte slots per plane
  constexpr int STAGE = 3 * PA + 3 * PB;
  constexpr int BK = 16 * KG;
  static_assert(TM >= 1 && TN >= 1 && BM == 32 * TM * WGM && BN == 32 * TN * WGN, "wave tiling");
  static_assert(2 * STAGE * 4 >= WGM * BN, "epilogue reduction buffer fits the staging LDS");
  constexpr bool AKC = MODE != 2, BKC = MODE == 0 || MODE == 3 || MODE == 4;
  constexpr int SCA = (AKC || (IMG & 2)) ? 0 : X6StageT<BM, KG, 64 * WGM * WGN>::SCRATCH;
  constexpr bool AIMG = (IMG & 2) != 0, BIMG = (IMG & 1) != 0;
  static_assert(IMG == 0 || MODE == 0 || MODE == 1 || MODE == 2 || (MODE == 4 && IMG == 1),
                "images: forward, input-grad, split-K epilogues (the split-K forward: B only)");
  static_assert(MODE != 2 || IMG == 0 || IMG == 3, "split-K: both operands as images");
  constexpr int SCB = (BKC || BIMG) ? 0 : X6StageT<BN, KG, 64 * WGM * WGN>::SCRATCH;
  constexpr int SCS = (SCA + SCB + 3) / 4;  // scratch in 16-byte slots, after the two stages
  __shared__ __attribute__((aligned(16))) bf16x8 lds[2 * STAGE + SCS];
  const GemmArgs& g = xa.g;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const unsigned nb = gridDim.x;
  unsigned L = blockIdx.x;
  if ((nb & 7u) == 0) L = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
  if ((int64_t)L >= g.tiles * xa.slices) return;
  const int slice = (int)((int64_t)L % xa.slices);
  const int64_t tile = (int64_t)L / xa.slices;
  const int64_t tm_idx = tile / g.tiles_n;
  const int64_t m0 = tm_idx * BM;
  const int n0 = (int)(tile % g.tiles_n) * BN;
  const int wm0 = (wave % WGM) * (32 * TM), wn0 = (wave / WGM) * (32 * TN);
  const int64_t mmax = g.M - 1;
  const int nmax = g.N - 1;
  constexpr bool SPLITK = MODE == 2 || MODE == 4;
  const int64_t kbeg = SPLITK ? (int64_t)slice * xa.kslice : 0;
  const int64_t kend = SPLITK ? min<int64_t>((int64_t)g.K, kbeg + xa.kslice) : g.K;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; m++)
#pragma unroll
    for (int n = 0; n < TN; n++) acc[m][n] = (f32x16)0.f;

  X6Op<BM, KG, NT, AKC, VEC> sa;
  X6Op<BN, KG, NT, BKC, VEC> sb;
  constexpr bool AP = APF && IMG == 1 && AKC;
  X6Op<BM, KG, NT, AKC, VEC> sa2;  // AP: A's second register set
  float* scA = reinterpret_cast<float*>(lds + 2 * STAGE);
  float* scB = scA + SCA;
  const int64_t nk = kend - kbeg;
  const int64_t kfull = kbeg + (nk & ~(int64_t)(BK - 1));
  const int nchunks = (int)((nk + BK - 1) / BK);
  // image chunk c (relative to kbeg) of an operand with R block rows from row r0: 3 planes x KG
  // chunk slices x R/32 units of 1 KB, one LDS-DMA instruction each, spread over the waves
  const int64_t cabs0 = kbeg / 16;
  auto dma = [&](auto RC, const float* img, int64_t pitch, int64_t r0, int c, bf16x8* dst) {
    constexpr int R = decltype(RC)::value, U = R / 32, PR = R * 2 * KG;
    const bf16x8* base = reinterpret_cast<const bf16x8*>(img) + r0 * 2 + lane;
    for (int q = wave; q < 3 * KG * U; q += WGM * WGN) {
      const int u = q % U, kg = (q / U) % KG, p = q / (U * KG);
      const bf16x8* src = base + ((cabs0 + (int64_t)c * KG + kg) * 3 + p) * pitch + u * 64;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + p * PR + kg * R * 2 + u * 64),
                                       16, 0, 0);
    }
  };
  auto dma_all = [&](int c, bf16x8* S) {
    if (AIMG) dma(std::integral_constant<int, BM>(), g.A, g.lda, m0, c, S);
    if (BIMG) dma(std::integral_constant<int, BN>(), g.B, g.ldb, n0, c, S + 3 * PA);
  };
  auto load = [&](int64_t kc) {
    const bool tail = kc + BK > kfull;
    if (!AIMG) sa.load(g.A, g.lda, m0, mmax, kc, kend, tail, tid);
    if (!BIMG) sb.load(g.B, g.ldb, n0, nmax, kc, kend, tail, tid);
  };
  auto store = [&](bf16x8* S) {
    if (!AIMG) {
      if (AKC) sa.kc.store(S, tid);
      else sa.rt.to_scratch(scA, tid);
    }
    if (!BIMG) {
      if (BKC) sb.kc.store(S + 3 * PA, tid);
      else sb.rt.to_scratch(scB, tid);
    }
    if ((!AKC && !AIMG) || (!BKC && !BIMG)) {
      __syncthreads();
      if (!AKC && !AIMG) sa.rt.to_planes(S, scA, tid);
      if (!BKC && !BIMG) sb.rt.to_planes(S + 3 * PA, scB, tid);
    }
  };
  auto mfma_chunk = [&](const bf16x8* cur) {
#pragma unroll
    for (int kg = 0; kg < KG; kg++) {
      bf16x8 a[3][TM], b[3][TN];
#pragma unroll
      for (int p = 0; p < 3; p++) {
#pragma unroll
        for (int m = 0; m < TM; m++) a[p][m] = cur[p * PA + x6_slot(BM, kg, wm0 + 32 * m + i, h)];
#pragma unroll
        for (int n = 0; n < TN; n++) b[p][n] = cur[3 * PA + p * PB + x6_slot(BN, kg, wn0 + 32 * n + i, h)];
      }
#pragma unroll
      for (int m = 0; m < TM; m++)
#pragma unroll
        for (int n = 0; n < TN; n++) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][m], b[0][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][m], b[1][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[2][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][m], b[0][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[1][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[0][n], acc[m][n], 0, 0, 0);
        }
    }
  };
  if (AP) {
    // chunk j's A in set j & 1: chunk c + 2 loads into the set chunk c left at the top of
    // iteration c, chunk c + 1 (loaded one iteration earlier) is split into LDS at its bottom
    auto loadA = [&](auto& S, int64_t kc) { S.load(g.A, g.lda, m0, mmax, kc, kend, kc + BK > kfull, tid); };
    if (nchunks > 0) {
      dma_all(0, lds);
      loadA(sa, kbeg);
      sa.kc.store(lds, tid);
      if (nchunks > 1) loadA(sa2, kbeg + BK);
    }
    __syncthreads();
    auto body = [&](int c, auto& L, auto& H) {
      const bf16x8* cur = lds + (c & 1) * STAGE;
      bf16x8* nxt = lds + ((c + 1) & 1) * STAGE;
      const bool more = c + 1 < nchunks;
      if (more) dma_all(c + 1, nxt);
      if (c + 2 < nchunks) loadA(L, kbeg + (int64_t)(c + 2) * BK);
      mfma_chunk(cur);
      if (more) H.kc.store(nxt, tid);
      __syncthreads();
    };
    for (int c = 0; c < nchunks; c += 2) {
      body(c, sa, sa2);
      if (c + 1 < nchunks) body(c + 1, sa2, sa);
    }
  } else {
  if (nchunks > 0) {
    if (IMG) dma_all(0, lds);
    if (IMG != 3) {
      load(kbeg);
      store(lds);
    }
  }
  __syncthreads();
  for (int c = 0; c < nchunks; c++) {
    const bf16x8* cur = lds + (c & 1) * STAGE;
    bf16x8* nxt = lds + ((c + 1) & 1) * STAGE;
    const bool more = c + 1 < nchunks;
    if (more) {
      if (IMG) dma_all(c + 1, nxt);
      if (IMG != 3) load(kbeg + (int64_t)(c + 1) * BK);
    }
#pragma unroll
    for (int kg = 0; kg < KG; kg++) {
      bf16x8 a[3][TM], b[3][TN];
#pragma unroll
      for (int p = 0; p < 3; p++) {
#pragma unroll
        for (int m = 0; m < TM; m++) a[p][m] = cur[p * PA + x6_slot(BM, kg, wm0 + 32 * m + i, h)];
#pragma unroll
        for (int n = 0; n < TN; n++) b[p][n] = cur[3 * PA + p * PB + x6_slot(BN, kg, wn0 + 32 * n + i, h)];
      }
#pragma unroll
      for (int m = 0; m < TM; m++)
#pragma unroll
        for (int n = 0; n < TN; n++) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][m], b[0][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][m], b[1][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[2][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][m], b[0][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[1][n], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[0][n], acc[m][n], 0, 0, 0);
        }
    }
    if (more && IMG != 3) store(nxt);
    __syncthreads();
  }
  }

  // epilogue (epi_forward / epi_input_grad)
  if (MODE == 0 || SPLITK) {
    float* Cs = g.C + (SPLITK ? (int64_t)slice * xa.cstride : 0);  // mode 3 takes the input-grad epilogue
    int64_t ldcs = g.ldc;
    int cshift = 0;
    const float* bs = g.bias;
    if (MODE == 0 && g.nsplit > 0 && n0 >= g.nsplit) {  // block-uniform: the split is a multiple of BN
      Cs = g.C2;
      ldcs = g.ldc2;
      cshift = g.nsplit;
      bs = g.bias2;
    }
    if (MODE == 0 && g.bias) epi_forward<TM, TN, MODE == 0 && ELU, true>(acc, g, Cs, m0 + wm0, n0 + wn0, i, h, ldcs, cshift, bs);
    else epi_forward<TM, TN, MODE == 0 && ELU, false>(acc, g, Cs, m0 + wm0, n0 + wn0, i, h, ldcs, cshift, bs);
  } else {
    float* red = reinterpret_cast<float*>(lds);  // [WGM][BN] column partials of the waves along M
    float cs[TN];
    epi_input_grad<TM, TN, ELU>(acc, g, m0 + wm0, n0 + wn0, i, h, cs);
#pragma unroll
    for (int n = 0; n < TN; n++) {
      const int cl = wn0 + 32 * n + i;
      cs[n] += __shfl_xor(cs[n], 32);
      if (h == 0) red[(wave % WGM) * BN + cl] = cs[n];
    }
    if (g.colpart) {
      __syncthreads();
      for (int c = tid; c < BN; c += NT) {
        if (n0 + c <= nmax) {
          float sum = 0.f;
#pragma unroll
          for (int w = 0; w < WGM; w++) sum += red[w * BN + c];
          g.colpart[tm_idx * g.N + n0 + c] = sum;
        }
      }
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int KG, bool VEC, int MODE, bool ELU, int IMG = 0, bool APF = false>
__global__ void __launch_bounds__(64 * WGM * WGN) k_gemm_x6(GemmX6Args xa) {
  gemm_x6_body<BM, BN, WGM, WGN, KG, VEC, MODE, ELU, IMG, APF>(xa);
}

// The same kernel compiled for OCC waves per SIMD (amdgpu_waves_per_eu: the register allocation
// held to 512 / OCC): a 256 x 128 tile on 8 waves uses 138 registers as k_gemm_x6, i.e. one block
// per CU, so a 480-block grid runs 1.875 dispatch rounds; at <= 128 registers (OCC 4) two blocks
// share a CU (LDS 2 x 72 KB) and the grid is one round
template <int BM, int BN, int WGM, int WGN, int KG, bool VEC, int MODE, bool ELU, int IMG = 0, bool APF = false,
          int OCC = 4>
__global__ void __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(OCC)))
k_gemm_x6_occ(GemmX6Args xa) {
  gemm_x6_body<BM, BN, WGM, WGN, KG, VEC, MODE, ELU, IMG, APF>(xa);
}

// Operand images of the bf16-split kernels, a list of operands in one launch.  An operand X with
// R rows (the product's M or N side) and reduction length K: element (r, k) = P[r ld + k]
// (trans 0: k-contiguous rows — W of the forward, activations, gradients as the A side) or
// P[k ld + r] (trans 1: reduction-major — W [K, N] of the input grad, the weight gradient's
// row-major gh / x).  Layout: chunks of 16 k (count rounded up to even, so 32-deep tiles read whole
// pairs), per chunk three planes (x0, x1, x2 of the exact split), per plane the rows padded to a
// multiple of 256, row r's 8-k half h at 16-byte slot (r / 32 * 2 + h) * 32 + r % 32 — the LDS
// fragment order of every tile (32-row units of 1 KB).  Zero past R and K.  Block (job, chunk,
// 128-row group), thread (row r, half h).
constexpr int IMG_MAX = 16;
struct ImageJobs {
  const float* P[IMG_MAX];
  bf16x8* img[IMG_MAX];
  int64_t ld[IMG_MAX], pitch[IMG_MAX];
  int trans[IMG_MAX], R[IMG_MAX], K[IMG_MAX], groups[IMG_MAX];
  int block0[IMG_MAX + 1];
  int njobs;
};

__host__ __device__ inline int64_t img_rows(int64_t R) { return (R + 255) / 256 * 256; }
__host__ __device__ inline int64_t img_chunks(int64_t K) { return (K + 31) / 32 * 2; }

__global__ void __launch_bounds__(256) k_x6_image_jobs(ImageJobs J) {
  const int bid = blockIdx.x;
  int j = 0;
  while (j + 1 < J.njobs && bid >= J.block0[j + 1]) j++;
  const int lb = bid - J.block0[j];
  const int grp = lb % J.groups[j], c = lb / J.groups[j];
  const int r = grp * 128 + (threadIdx.x & 127), h = threadIdx.x >> 7;
  const float* __restrict__ P = J.P[j];
  const int64_t ld = J.ld[j];
  const int R = J.R[j], K = J.K[j];
  const int k0 = c * 16 + 8 * h;
  float v[8];
  if (J.trans[j]) {
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = (r < R && k0 + q < K) ? P[(int64_t)(k0 + q) * ld + r] : 0.f;
  } else if (r < R && k0 + 8 <= K && ld % 4 == 0 && ((uintptr_t)P & 15) == 0) {
    const float4 a = *reinterpret_cast<const float4*>(P + (int64_t)r * ld + k0);
    const float4 b = *reinterpret_cast<const float4*>(P + (int64_t)r * ld + k0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = (r < R && k0 + q < K) ? P[(int64_t)r * ld + k0 + q] : 0.f;
  }
  bf16x8 x0, x1, x2;
  split3x8(v, x0, x1, x2);
  const int64_t pitch = J.pitch[j];
  bf16x8* base = J.img[j] + (int64_t)c * 3 * pitch + (r / 32 * 2 + h) * 32 + r % 32;
  base[0] = x0;
  base[pitch] = x1;
  base[2 * pitch] = x2;
}

template <int BM, int BN, int WGM, int WGN, int KG, bool APF = false, int OCC = 0>
int launch_x6_img(int mode, int img, GemmX6Args xa, bool vec, bool elu, hipStream_t s) {
  GemmArgs& g = xa.g;
  g.tiles_n = (g.N + BN - 1) / BN;
  const int64_t tiles_m = (g.M + BM - 1) / BM;
  g.tiles = tiles_m * g.tiles_n;
  if (mode != 2 && mode != 4) xa.slices = 1;
  if (g.tiles * xa.slices > 0x7fffffff) return HG_ERR_ARG;
  const dim3 grid((unsigned)(g.tiles * xa.slices)), block(64 * WGM * WGN);
#define HG_X6I(V, MD, E, I)                                                                                      \
  do {                                                                                                             \
    if constexpr (OCC > 0) hipLaunchKernelGGL((k_gemm_x6_occ<BM, BN, WGM, WGN, KG, V, MD, E, I, APF, OCC>), grid, block, 0, s, xa); \
    else hipLaunchKernelGGL((k_gemm_x6<BM, BN, WGM, WGN, KG, V, MD, E, I, APF>), grid, block, 0, s, xa);             \
  } while (0)
  if (mode == 2) {
    HG_X6I(false, 2, false, 3);
  } else if (mode == 4) {  // the split-K forward's slices with W as the image
    if (vec) HG_X6I(true, 4, false, 1);
    else HG_X6I(false, 4, false, 1);
  } else if (img == 3) {
    if (mode == 0) {
      if (elu) HG_X6I(false, 0, true, 3);
      else HG_X6I(false, 0, false, 3);
    } else {
      if (elu) HG_X6I(false, 1, true, 3);
      else HG_X6I(false, 1, false, 3);
    }
  } else if (mode == 0) {
    if (vec && elu) HG_X6I(true, 0, true, 1);
    else if (vec) HG_X6I(true, 0, false, 1);
    else if (elu) HG_X6I(false, 0, true, 1);
    else HG_X6I(false, 0, false, 1);
  } else {
    if (vec && elu) HG_X6I(true, 1, true, 1);
    else if (vec) HG_X6I(true, 1, false, 1);
    else if (elu) HG_X6I(false, 1, true, 1);
    else HG_X6I(false, 1, false, 1);
  }
#undef HG_X6I
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

int x6_img_dispatch(int tile, int mode, int img, GemmX6Args xa, bool vec, bool elu, hipStream_t s) {
  switch (tile) {
    case 20: return launch_x6_img<128, 128, 2, 2, 1>(mode, img, xa, vec, elu, s);
    case 21: return launch_x6_img<128, 128, 2, 4, 1>(mode, img, xa, vec, elu, s);
    case 22: return launch_x6_img<128, 64, 2, 2, 1>(mode, img, xa, vec, elu, s);
    case 23: return launch_x6_img<64, 64, 2, 2, 1>(mode, img, xa, vec, elu, s);
    case 24: return launch_x6_img<128, 128, 2, 2, 2>(mode, img, xa, vec, elu, s);
    case 25: return launch_x6_img<256, 128, 4, 2, 1>(mode, img, xa, vec, elu, s);
    case 26: return launch_x6_img<128, 128, 2, 4, 2>(mode, img, xa, vec, elu, s);
    case 27: return launch_x6_img<128, 256, 2, 4, 1>(mode, img, xa, vec, elu, s);
    case 28: return launch_x6_img<64, 256, 2, 4, 1>(mode, img, xa, vec, elu, s);
    // 29: tile 23 with A two chunks ahead (APF; B-image form only).  The same variant of tiles 20,
    // 21, 22 and 28 measured slower on every routed shape (profiles/r4_gemm/x6_apf_probe.jsonl)
    case 29: return launch_x6_img<64, 64, 2, 2, 1, true>(mode, img, xa, vec, elu, s);
    // 30: tile 25 at two blocks per CU; 31: tile 22 at four (k_gemm_x6_occ, 4 waves per SIMD)
    case 30: return launch_x6_img<256, 128, 4, 2, 1, false, 4>(mode, img, xa, vec, elu, s);
    case 31: return launch_x6_img<128, 64, 2, 2, 1, false, 4>(mode, img, xa, vec, elu, s);
    // 32: tile 21 (128 x 128 on 8 waves, 90 registers: two blocks per CU) at three (6 waves per SIMD)
    case 32: return launch_x6_img<128, 128, 2, 4, 1, false, 6>(mode, img, xa, vec, elu, s);
    default: return launch_x6_img<64, 128, 2, 2, 1>(mode, img, xa, vec, elu, s);  // 19
  }
}

template <int BM, int BN, int WGM, int WGN, int KG>
int launch_x6(int mode, GemmX6Args xa, bool vec, bool elu, hipStream_t s) {
  GemmArgs& g = xa.g;
  g.tiles_n = (g.N + BN - 1) / BN;
  const int64_t tiles_m = (g.M + BM - 1) / BM;
  g.tiles = tiles_m * g.tiles_n;
  if (mode != 2 && mode != 4) xa.slices = 1;
  if (g.tiles * xa.slices > 0x7fffffff) return HG_ERR_ARG;
  const dim3 grid((unsigned)(g.tiles * xa.slices)), block(64 * WGM * WGN);
#define HG_X6(V, MD, E) hipLaunchKernelGGL((k_gemm_x6<BM, BN, WGM, WGN, KG, V, MD, E>), grid, block, 0, s, xa)
  if (mode == 0) {
    if (vec && elu) HG_X6(true, 0, true);
    else if (vec) HG_X6(true, 0, false);
    else if (elu) HG_X6(false, 0, true);
    else HG_X6(false, 0, false);
  } else if (mode == 1) {
    if (vec && elu) HG_X6(true, 1, true);
    else if (vec) HG_X6(true, 1, false);
    else if (elu) HG_X6(false, 1, true);
    else HG_X6(false, 1, false);
  } else if (mode == 3) {
    if (vec && elu) HG_X6(true, 3, true);
    else if (vec) HG_X6(true, 3, false);
    else if (elu) HG_X6(false, 3, true);
    else HG_X6(false, 3, false);
  } else if (mode == 4) {
    if (vec) HG_X6(true, 4, false);
    else HG_X6(false, 4, false);
  } else {
    HG_X6(false, 2, false);
  }
#undef HG_X6
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

constexpr int NTILES = 29;  // 29: tile 23 with A two chunks ahead (image entry)
constexpr int NTILES_IMG = 32;  // the image entries also take 30 / 31 / 32: tiles 25 / 22 / 21 at more waves per SIMD
// block rows of a tile id (the column-partial row count of mode 1)
int tile_bm(int tile) {
  if (tile == 25 || tile == 30) return 256;
  return (tile <= 2 || (tile >= 8 && tile <= 10) || tile == 12 || tile == 13 || tile == 16 || tile == 17 ||
          (tile >= 20 && tile <= 22) || tile == 24 || tile == 26 || tile == 27 || tile == 31 || tile == 32)
             ? 128
             : 64;
}

// ---------------------------------------------------------------------------------------------
// Weight gradient on the bf16 matrix cores with LDS transpose reads (round 4):
//   C_s[m][n] = sum_{r in slice s} A[r][m] B[r][n]     A = gh [R, M], B = x [R, N], both row-major
// (the reduction runs over the ROWS of both operands, as dW = gh^T x).  Each 16-row chunk of both
// operands is staged exactly as it lies in memory: coalesced float4 row segments -> registers ->
// the exact three-term bf16 split (v_cvt_pk_bf16_f32 pairs) -> three row-major bf16 planes in LDS
// ([16 rows][cols], rows padded by 64 B so a transposed read's four rows fall on disjoint banks).
// ds_read_b64_tr_b16 then delivers the MFMA operand directly: for the 32x32x16 operand, lane
// (i, h) needs 8 consecutive reduction rows 8h..8h+7 of column i, i.e. two transposed reads of 4
// rows x 16 columns per 16-lane group (lane 4q + p addresses row q, columns 4p..4p+3; lane i of
// the group receives column i).  No transposing staging pass, each element split once per block.
// The six partial products as k_gemm_x6 (smallest first).  Split-K: slice s covers kslice rows and
// writes C + s cstride; the slices are summed in fixed order by the column-sum launch.
struct WgradArgs {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc, cstride;
  int M, N;
  int64_t R, kslice;
  int slices, tiles_n;
  int64_t tiles;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t bf16_pair(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ f32x2 bf16_pair_f32(uint32_t u) {
  f32x2 r;
  r[0] = __uint_as_float(u << 16);
  r[1] = __uint_as_float(u & 0xffff0000u);
  return r;
}
// exact split of 4 consecutive values into three planes of 4 bf16 (8 bytes each)
__device__ __forceinline__ void split3x4(const float v[4], uint2& p0, uint2& p1, uint2& p2) {
  f32x2 a = {v[0], v[1]}, b = {v[2], v[3]};
  const uint32_t a0 = bf16_pair(a), b0 = bf16_pair(b);
  a -= bf16_pair_f32(a0);
  b -= bf16_pair_f32(b0);
  const uint32_t a1 = bf16_pair(a), b1 = bf16_pair(b);
  a -= bf16_pair_f32(a1);
  b -= bf16_pair_f32(b1);
  p0 = make_uint2(a0, b0);
  p1 = make_uint2(a1, b1);
  p2 = make_uint2(bf16_pair(a), bf16_pair(b));
}

// one operand's 16-row chunk: COLS columns from col0, rows r0.. (rows at or past rend and columns at
// or past ncols read 0); items (row, float4 column group), consecutive threads along a row
template <int COLS, int NT>
struct TrStage {
  static constexpr int ITEMS = 16 * (COLS / 4);
  static constexpr int IPT = (ITEMS + NT - 1) / NT;
  static constexpr int PITCH = COLS * 2 + 64;  // bytes per LDS row of one plane
  static constexpr int PLANE = 16 * PITCH;
  float v[IPT][4];
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int64_t r0, int64_t rend, int col0,
                                       int ncols, int tid) {
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int idx = tid + j * NT;
      if (ITEMS % NT != 0 && idx >= ITEMS) break;
      const int row = idx / (COLS / 4), c = col0 + 4 * (idx % (COLS / 4));
      const int64_t r = r0 + row;
      const float* p = P + r * ld + c;
      if (r < rend && c + 3 < ncols) {
        const f32x4u x = *reinterpret_cast<const f32x4u*>(p);
        v[j][0] = x[0]; v[j][1] = x[1]; v[j][2] = x[2]; v[j][3] = x[3];
      } else {
#pragma unroll
        for (int e = 0; e < 4; e++) v[j][e] = (r < rend && c + e < ncols) ? p[e] : 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(char* __restrict__ S, int tid) const {
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int idx = tid + j * NT;
      if (ITEMS % NT != 0 && idx >= ITEMS) break;
      const int row = idx / (COLS / 4), c4 = idx % (COLS / 4);
      uint2 x0, x1, x2;
      split3x4(v[j], x0, x1, x2);
      char* d = S + row * PITCH + 8 * c4;
      *reinterpret_cast<uint2*>(d) = x0;
      *reinterpret_cast<uint2*>(d + PLANE) = x1;
      *reinterpret_cast<uint2*>(d + 2 * PLANE) = x2;
    }
  }
};

// the 32x32x16 operand of columns c0 + 0..31 of a staged plane (rows 0..15 of the chunk)
template <int PITCH>
__device__ __forceinline__ bf16x8 tr_operand(const char* __restrict__ plane, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const char* a = plane + (8 * (g >> 1) + q) * PITCH + 2 * (c0 + 16 * (g & 1) + 4 * p);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * PITCH));
  const short e[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, e);
}

template <int WGM, int WGN, int TM, int TN, int PF>
__global__ void __launch_bounds__(64 * WGM * WGN) k_wgrad_tr(WgradArgs w) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int BM = 32 * TM * WGM, BN = 32 * TN * WGN;
  typedef TrStage<BM, NT> SA;
  typedef TrStage<BN, NT> SB;
  constexpr int STAGE = 3 * SA::PLANE + 3 * SB::PLANE;  // bytes
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const unsigned nb = gridDim.x;
  unsigned L = blockIdx.x;
  if ((nb & 7u) == 0) L = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
  if ((int64_t)L >= w.tiles * w.slices) return;
  // the tiles of one slice are consecutive (one XCD's L2 serves the slice's rows to all of them)
  const int slice = (int)((int64_t)L / w.tiles);
  const int64_t tile = (int64_t)L % w.tiles;
  const int m0 = (int)(tile / w.tiles_n) * BM, n0 = (int)(tile % w.tiles_n) * BN;
  const int wm0 = (wave % WGM) * (32 * TM), wn0 = (wave / WGM) * (32 * TN);
  const int64_t kbeg = (int64_t)slice * w.kslice;
  const int64_t kend = min<int64_t>(w.R, kbeg + w.kslice);
  const int nchunks = kend > kbeg ? (int)((kend - kbeg + 15) / 16) : 0;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; m++)
#pragma unroll
    for (int n = 0; n < TN; n++) acc[m][n] = (f32x16)0.f;

  // one chunk: the global loads of chunk c + PF into (la, lb), the MFMAs on stage c & 1, the split
  // + LDS store of chunk c + 1 from (ha, hb) into the other stage, one barrier
  auto step = [&](int c, SA& la, SB& lb, const SA& ha, const SB& hb) {
    const char* cur = lds + (c & 1) * STAGE;
    char* nxt = lds + ((c + 1) & 1) * STAGE;
    if (c + PF < nchunks) {
      const int64_t r0 = kbeg + (int64_t)(c + PF) * 16;
      la.load(w.A, w.lda, r0, kend, m0, w.M, tid);
      lb.load(w.B, w.ldb, r0, kend, n0, w.N, tid);
    }
    bf16x8 a[3][TM], b[3][TN];
#pragma unroll
    for (int p = 0; p < 3; p++) {
#pragma unroll
      for (int m = 0; m < TM; m++) a[p][m] = tr_operand<SA::PITCH>(cur + p * SA::PLANE, wm0 + 32 * m, lane);
#pragma unroll
      for (int n = 0; n < TN; n++)
        b[p][n] = tr_operand<SB::PITCH>(cur + 3 * SA::PLANE + p * SB::PLANE, wn0 + 32 * n, lane);
    }
#pragma unroll
    for (int m = 0; m < TM; m++)
#pragma unroll
      for (int n = 0; n < TN; n++) {
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][m], b[0][n], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][m], b[1][n], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[2][n], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][m], b[0][n], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[1][n], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][m], b[0][n], acc[m][n], 0, 0, 0);
      }
    if (c + 1 < nchunks) {
      ha.store(nxt, tid);
      hb.store(nxt + 3 * SA::PLANE, tid);
    }
    __syncthreads();
  };
  SA sa0, sa1;
  SB sb0, sb1;
  if (nchunks > 0) {
    sa0.load(w.A, w.lda, kbeg, kend, m0, w.M, tid);
    sb0.load(w.B, w.ldb, kbeg, kend, n0, w.N, tid);
    sa0.store(lds, tid);
    sb0.store(lds + 3 * SA::PLANE, tid);
    if (PF == 2 && nchunks > 1) {
      sa1.load(w.A, w.lda, kbeg + 16, kend, m0, w.M, tid);
      sb1.load(w.B, w.ldb, kbeg + 16, kend, n0, w.N, tid);
    }
  }
  __syncthreads();
  if (PF == 1) {
    for (int c = 0; c < nchunks; c++) step(c, sa0, sb0, sa0, sb0);
  } else {
    // two register sets: chunk c + 1 waits in one while chunk c + 2 loads into the other
    for (int c = 0; c < nchunks; c += 2) {
      step(c, sa0, sb0, sa1, sb1);
      if (c + 1 < nchunks) step(c + 1, sa1, sb1, sa0, sb0);
    }
  }
  // epilogue: acc register q of a 32x32 tile is row (q & 3) + 8 (q >> 2) + 4h, column i
  float* Cs = w.C + (int64_t)slice * w.cstride;
#pragma unroll
  for (int n = 0; n < TN; n++) {
    const int col = n0 + wn0 + 32 * n + i;
    if (col >= w.N) continue;
#pragma unroll
    for (int m = 0; m < TM; m++)
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int row = m0 + wm0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (row < w.M) Cs[(int64_t)row * w.ldc + col] = acc[m][n][q];
      }
  }
}

template <int WGM, int WGN, int TM, int TN, int PF = 1>
int launch_wgrad_tr(WgradArgs w, hipStream_t s) {
  constexpr int BM = 32 * TM * WGM, BN = 32 * TN * WGN;
  w.tiles_n = (w.N + BN - 1) / BN;
  w.tiles = (int64_t)((w.M + BM - 1) / BM) * w.tiles_n;
  if (w.tiles * w.slices > 0x7fffffff) return HG_ERR_ARG;
  hipLaunchKernelGGL((k_wgrad_tr<WGM, WGN, TM, TN, PF>), dim3((unsigned)(w.tiles * w.slices)), dim3(64 * WGM * WGN), 0, s, w);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

constexpr int WGRAD_TR0 = 40, WGRAD_TR1 = 54;  // tile ids of k_wgrad_tr (hg_gemm_f32_wgrad only)

}  // namespace

extern "C" int64_t hg_gemm_x6_image_bytes(int64_t rows, int64_t K) {
  if (rows <= 0 || K <= 0 || rows > 0x7fffffff || K > 0x7fffffff) return -1;
  return img_chunks(K) * 3 * img_rows(rows) * 2 * 16;
}

extern "C" int hg_gemm_x6_image_jobs_pitched(const float* const* P, const int64_t* ld, const int* trans,
                                             const int64_t* rows, const int64_t* K, void* const* img,
                                             const int64_t* pitch_rows, int njobs, void* stream);

extern "C" int hg_gemm_x6_image_jobs(const float* const* P, const int64_t* ld, const int* trans, const int64_t* rows,
                                     const int64_t* K, void* const* img, int njobs, void* stream) {
  return hg_gemm_x6_image_jobs_pitched(P, ld, trans, rows, K, img, nullptr, njobs, stream);
}

// pitch_rows (nullable; entry <= 0: the job's own rows): the row count of the image a job writes
// into, so several jobs fill the row bands of ONE image (job j's img = the image + its first row
// x 32 bytes): the image of the rows stacked, e.g. two layers' weights that read the same input as
// one [n_a + n_b, K] operand.  Every job writes img_rows(its rows) rows (zero past them), so the
// bands of one image must come as one chain of consecutive jobs (same pitch_rows and K, each band
// starting where the previous one ends) whose rows sum to pitch_rows, every band but the last a
// multiple of 256 rows: then no band's zero padding lands on the next band and the last one's ends
// at img_rows(pitch_rows), inside the image (a 480 + 32 split would race on rows 480..511 and write
// past the image).
extern "C" int hg_gemm_x6_image_jobs_pitched(const float* const* P, const int64_t* ld, const int* trans,
                                             const int64_t* rows, const int64_t* K, void* const* img,
                                             const int64_t* pitch_rows, int njobs, void* stream) {
  if (njobs <= 0) return HG_OK;
  if (njobs > IMG_MAX || !P || !ld || !trans || !rows || !K || !img) return HG_ERR_ARG;
  ImageJobs J;
  J.njobs = njobs;
  int64_t blocks = 0;
  for (int j = 0; j < njobs; j++) {
    if (!P[j] || !img[j] || rows[j] <= 0 || K[j] <= 0 || rows[j] > 0x7fffffff || K[j] > 0x7fffffff ||
        (trans[j] != 0 && trans[j] != 1))
      return HG_ERR_ARG;
    if ((trans[j] == 0 && ld[j] < K[j]) || (trans[j] == 1 && ld[j] < rows[j])) return HG_ERR_ARG;
    if ((uintptr_t)P[j] % 4 || (uintptr_t)img[j] % 16) return HG_ERR_ARG;
    J.P[j] = P[j];
    J.img[j] = reinterpret_cast<bf16x8*>(img[j]);
    J.ld[j] = ld[j];
    const int64_t prow = pitch_rows && pitch_rows[j] > 0 ? pitch_rows[j] : rows[j];
    if (prow < rows[j] || prow > 0x7fffffff) return HG_ERR_ARG;
    J.pitch[j] = img_rows(prow) * 2;
    J.trans[j] = trans[j];
    J.R[j] = (int)rows[j];
    J.K[j] = (int)K[j];
    J.groups[j] = (int)(img_rows(rows[j]) / 128);
    J.block0[j] = (int)blocks;
    blocks += img_chunks(K[j]) * J.groups[j];
    if (blocks > (int64_t)1 << 30) return HG_ERR_ARG;
  }
  J.block0[njobs] = (int)blocks;
  for (int j = 0; j < njobs;) {  // band chains (see above)
    const int64_t prow = pitch_rows && pitch_rows[j] > 0 ? pitch_rows[j] : rows[j];
    int64_t sum = rows[j];
    int e = j + 1;
    while (e < njobs && pitch_rows && pitch_rows[e] == prow && K[e] == K[j] && sum < prow &&
           (uintptr_t)img[e] == (uintptr_t)img[e - 1] + (uintptr_t)(32 * rows[e - 1])) {
      sum += rows[e];
      e++;
    }
    if (sum != prow) return HG_ERR_ARG;
    for (int b = j; b + 1 < e; b++)
      if (rows[b] % 256) return HG_ERR_ARG;
    j = e;
  }
  hipLaunchKernelGGL(k_x6_image_jobs, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, J);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

extern "C" int hg_gemm_f32_img(int mode, const float* A, int64_t lda, const void* Aimg, const void* Bimg,
                               const float* bias, const float* Y, int64_t ldY, float* C, int64_t ldc, float* colpart,
                               int64_t M, int N, int K, int act, int tile, int64_t aimg_bytes, int64_t bimg_bytes,
                               void* stream) {
  if ((!A && !Aimg) || !Bimg || !C || M <= 0 || N <= 0 || K <= 0 || ldc < N || (mode != 0 && mode != 1) || act < 0 ||
      act > 1 || tile < 19 || tile > NTILES_IMG)
    return HG_ERR_ARG;
  if (!Aimg && lda < K) return HG_ERR_ARG;
  // the images must be the ones hg_gemm_x6_image_jobs builds for this product's shape
  if (bimg_bytes != hg_gemm_x6_image_bytes(N, K) || (Aimg && aimg_bytes != hg_gemm_x6_image_bytes(M, K)))
    return HG_ERR_ARG;
  if (mode == 1 && act == 1 && (!Y || ldY < N)) return HG_ERR_ARG;
  if ((!Aimg && (uintptr_t)A % 4) || (uintptr_t)Aimg % 16 || (uintptr_t)Bimg % 16 || (uintptr_t)C % 4)
    return HG_ERR_ARG;
  const bool vec = !Aimg && lda % 4 == 0 && (uintptr_t)A % 16 == 0;
  const float* a = Aimg ? reinterpret_cast<const float*>(Aimg) : A;
  const int64_t la = Aimg ? img_rows(M) * 2 : lda;
  GemmArgs g{a, la, reinterpret_cast<const float*>(Bimg), img_rows(N) * 2, bias, Y, ldY, C, ldc, colpart, M, N, K, 0, 0};
  GemmX6Args xa{g, 0, 0, 1};
  return x6_img_dispatch(tile, mode, Aimg ? 3 : 1, xa, vec, act == 1, (hipStream_t)stream);
}

extern "C" int hg_gemm_f32_img_split(const float* A, int64_t lda, const void* Bimg, const float* bias,
                                     const float* bias2, float* C, int64_t ldc, float* C2, int64_t ldc2, int nsplit,
                                     int64_t M, int N, int K, int act, int tile, int64_t bimg_bytes, void* stream) {
  if (!A || !Bimg || !C || !C2 || !bias != !bias2 || M <= 0 || N <= 0 || K <= 0 || nsplit <= 0 || nsplit >= N || nsplit % 256 ||
      ldc < nsplit || ldc2 < N - nsplit || lda < K || act < 0 || act > 1 || tile < 19 || tile > NTILES_IMG)
    return HG_ERR_ARG;
  if (bimg_bytes != hg_gemm_x6_image_bytes(N, K)) return HG_ERR_ARG;
  if ((uintptr_t)A % 4 || (uintptr_t)Bimg % 16 || (uintptr_t)C % 4 || (uintptr_t)C2 % 4) return HG_ERR_ARG;
  const bool vec = lda % 4 == 0 && (uintptr_t)A % 16 == 0;
  GemmArgs g{A, lda, reinterpret_cast<const float*>(Bimg), img_rows(N) * 2, bias, nullptr, 0, C, ldc, nullptr, M, N, K,
             0, 0, C2, ldc2, nsplit, bias2};
  GemmX6Args xa{g, 0, 0, 1};
  return x6_img_dispatch(tile, 0, 1, xa, vec, act == 1, (hipStream_t)stream);
}

extern "C" int hg_gemm_wgrad_img(const void* Aimg, const void* Bimg, float* C, int64_t ldc, int64_t cstride, int64_t M,
                                 int N, int64_t K, int slices, int tile, int64_t aimg_bytes, int64_t bimg_bytes,
                                 void* stream) {
  if (!Aimg || !Bimg || !C || M <= 0 || N <= 0 || K <= 0 || K > 0x7fffffff || ldc < N || slices < 1 || tile < 19 ||
      tile > NTILES)
    return HG_ERR_ARG;
  if (aimg_bytes != hg_gemm_x6_image_bytes(M, K) || bimg_bytes != hg_gemm_x6_image_bytes(N, K)) return HG_ERR_ARG;
  if (slices > 1 && cstride < M * (int64_t)ldc) return HG_ERR_ARG;
  if ((uintptr_t)Aimg % 16 || (uintptr_t)Bimg % 16 || (uintptr_t)C % 4) return HG_ERR_ARG;
  GemmArgs g{reinterpret_cast<const float*>(Aimg), img_rows(M) * 2, reinterpret_cast<const float*>(Bimg),
             img_rows(N) * 2, nullptr, nullptr, 0, C, ldc, nullptr, M, N, (int)K, 0, 0};
  // slices start on whole 32-deep chunk pairs of the images
  const int64_t kslice = ((K + slices - 1) / slices + 31) & ~(int64_t)31;
  GemmX6Args xa{g, kslice, cstride, slices};
  return x6_img_dispatch(tile, 2, 3, xa, false, false, (hipStream_t)stream);
}

extern "C" int hg_gemm_tile(int mode, int64_t M, int N, int K) {
  (void)mode;
  (void)K;
  // pipelined 128 x 64 tile on 8 waves while that gives >= 3 blocks per CU, else 64 x 64
  // (scripts/gemm_probe.py, profiles/r3_gemm)
  const int64_t t16 = ((M + 127) / 128) * ((N + 63) / 64);
  return t16 >= 768 ? 16 : 5;
}

extern "C" int64_t hg_gemm_colpart_rows(int64_t M, int tile) {
  if (tile < 1 || tile > NTILES_IMG) return -1;
  const int bm = tile_bm(tile);
  return (M + bm - 1) / bm;
}

extern "C" int hg_gemm_f32(int mode, const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                           const float* Y, int64_t ldY, float* C, int64_t ldc, float* colpart, int64_t M, int N, int K,
                           int act, int tile, void* stream) {
  // the occupancy tiles of the image entries run here (no image) as their base blocking: the same
  // products in the same order, so the same bits
  if (tile == 30) tile = 25;
  else if (tile == 31) tile = 22;
  else if (tile == 32) tile = 21;
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldc < N || mode < 0 || mode > 3 || mode == 2 ||
      act < 0 || act > 1 || tile < 1 || tile > NTILES)
    return HG_ERR_ARG;
  if (mode == 3 && tile < 19) return HG_ERR_ARG;  // the transposed-W input grad: bf16-split tiles only
  if ((mode == 0 || mode == 3) && ldb < K) return HG_ERR_ARG;
  if (mode == 1 && ldb < N) return HG_ERR_ARG;
  if ((mode == 1 || mode == 3) && act == 1 && (!Y || ldY < N)) return HG_ERR_ARG;
  if ((uintptr_t)A % 4 || (uintptr_t)B % 4 || (uintptr_t)C % 4) return HG_ERR_ARG;
  const bool vec = lda % 4 == 0 && (uintptr_t)A % 16 == 0 &&
                   (mode == 1 || (ldb % 4 == 0 && (uintptr_t)B % 16 == 0));
  GemmArgs g{A, lda, B, ldb, bias, Y, ldY, C, ldc, colpart, M, N, K, 0, 0};
  hipStream_t s = (hipStream_t)stream;
  const bool elu = act == 1;
  switch (tile) {  // <BM, BN, WGM, WGN, BK, LAY>
    case 1: return launch<128, 128, 2, 2, 32, 0>(mode, g, vec, elu, s);
    case 2: return launch<128, 64, 2, 2, 32, 0>(mode, g, vec, elu, s);
    case 3: return launch<64, 128, 2, 2, 32, 0>(mode, g, vec, elu, s);
    case 4: return launch<64, 64, 2, 2, 32, 0>(mode, g, vec, elu, s);
    case 5: return launch<64, 64, 2, 2, 32, 1>(mode, g, vec, elu, s);
    case 6: return launch<64, 64, 2, 2, 64, 0>(mode, g, vec, elu, s);
    case 7: return launch<64, 64, 2, 2, 64, 1>(mode, g, vec, elu, s);
    case 8: return launch<128, 64, 4, 2, 32, 1>(mode, g, vec, elu, s);
    case 9: return launch<128, 128, 2, 4, 32, 1>(mode, g, vec, elu, s);
    case 10: return launch<128, 64, 2, 2, 64, 1>(mode, g, vec, elu, s);
    case 11: return launch<64, 64, 2, 2, 16, 1>(mode, g, vec, elu, s);
    case 12: return launch<128, 128, 2, 4, 16, 1>(mode, g, vec, elu, s);
    case 13: return launch<128, 64, 4, 2, 16, 1>(mode, g, vec, elu, s);
    case 14: return launch<64, 128, 2, 2, 16, 1>(mode, g, vec, elu, s);
    case 15: return launch<64, 64, 2, 2, 32, 1, 1>(mode, g, vec, elu, s);
    case 16: return launch<128, 64, 4, 2, 32, 1, 1>(mode, g, vec, elu, s);
    case 17: return launch<128, 128, 2, 4, 32, 1, 1>(mode, g, vec, elu, s);
    case 18: return launch<64, 64, 2, 2, 16, 1, 1>(mode, g, vec, elu, s);
    default: break;
  }
  // tiles 20..26: the bf16-split (6-term) kernels, <BM, BN, WGM, WGN, KG>
  GemmX6Args xa{g, 0, 0, 1};
  switch (tile) {
    case 20: return launch_x6<128, 128, 2, 2, 1>(mode, xa, vec, elu, s);
    case 21: return launch_x6<128, 128, 2, 4, 1>(mode, xa, vec, elu, s);
    case 22: return launch_x6<128, 64, 2, 2, 1>(mode, xa, vec, elu, s);
    case 29:
    case 23: return launch_x6<64, 64, 2, 2, 1>(mode, xa, vec, elu, s);
    case 24: return launch_x6<128, 128, 2, 2, 2>(mode, xa, vec, elu, s);
    case 25: return launch_x6<256, 128, 4, 2, 1>(mode, xa, vec, elu, s);
    case 26: return launch_x6<128, 128, 2, 4, 2>(mode, xa, vec, elu, s);
    case 27: return launch_x6<128, 256, 2, 4, 1>(mode, xa, vec, elu, s);
    case 28: return launch_x6<64, 256, 2, 4, 1>(mode, xa, vec, elu, s);
    default: return launch_x6<64, 128, 2, 2, 1>(mode, xa, vec, elu, s);  // 19
  }
}

extern "C" int hg_gemm_f32_wgrad(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                                 int64_t cstride, int64_t M, int N, int64_t K, int slices, int kmajor, int tile,
                                 void* stream) {
  const bool tr = tile >= WGRAD_TR0 && tile <= WGRAD_TR1;
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || ldc < N || slices < 1 || (!tr && (tile < 19 || tile > 28)) ||
      K > 0x7fffffff || (kmajor != 0 && kmajor != 1) || (tr && (kmajor != 0 || M > 0x7fffffff)))
    return HG_ERR_ARG;
  if (kmajor == 0 && (lda < M || ldb < N)) return HG_ERR_ARG;
  if (kmajor == 1 && (lda < K || ldb < K)) return HG_ERR_ARG;
  if (slices > 1 && cstride < M * (int64_t)ldc) return HG_ERR_ARG;
  if ((uintptr_t)A % 4 || (uintptr_t)B % 4 || (uintptr_t)C % 4) return HG_ERR_ARG;
  const int64_t kslice = ((K + slices - 1) / slices + 15) & ~(int64_t)15;
  hipStream_t s = (hipStream_t)stream;
  if (tr) {
    // tiles 40..54: k_wgrad_tr <WGM, WGN, TM, TN, PF> (row-major operands, transposed LDS reads)
    WgradArgs w{A, lda, B, ldb, C, ldc, cstride, (int)M, N, K, kslice, slices, 0, 0};
    switch (tile) {
      case 40: return launch_wgrad_tr<4, 2, 2, 3>(w, s);  // 256 x 192, 8 waves
      case 41: return launch_wgrad_tr<4, 2, 2, 2>(w, s);  // 256 x 128, 8 waves
      case 42: return launch_wgrad_tr<2, 2, 2, 2>(w, s);  // 128 x 128, 4 waves
      case 43: return launch_wgrad_tr<2, 4, 2, 2>(w, s);  // 128 x 256, 8 waves
      case 44: return launch_wgrad_tr<2, 2, 2, 3>(w, s);  // 128 x 192, 4 waves
      case 45: return launch_wgrad_tr<4, 2, 1, 2>(w, s);  // 128 x 128, 8 waves
      case 46: return launch_wgrad_tr<2, 2, 1, 1>(w, s);  // 64 x 64, 4 waves
      case 47: return launch_wgrad_tr<2, 2, 1, 2>(w, s);  // 64 x 128, 4 waves
      case 48: return launch_wgrad_tr<2, 2, 2, 1>(w, s);  // 128 x 64, 4 waves
      // the same tiles with the global loads two chunks ahead (two register sets)
      case 49: return launch_wgrad_tr<4, 2, 2, 3, 2>(w, s);
      case 50: return launch_wgrad_tr<4, 2, 2, 2, 2>(w, s);
      case 51: return launch_wgrad_tr<2, 2, 2, 2, 2>(w, s);
      case 52: return launch_wgrad_tr<2, 2, 1, 1, 2>(w, s);
      case 53: return launch_wgrad_tr<2, 2, 1, 2, 2>(w, s);
      default: return launch_wgrad_tr<4, 2, 1, 2, 2>(w, s);  // 54
    }
  }
  GemmArgs g{A, lda, B, ldb, nullptr, nullptr, 0, C, ldc, nullptr, M, N, (int)K, 0, 0};
  GemmX6Args xa{g, kslice, cstride, slices};
  const int md = kmajor ? 4 : 2;
  const bool vec = kmajor && lda % 4 == 0 && ldb % 4 == 0 && (uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0;
  switch (tile) {
    case 20: return launch_x6<128, 128, 2, 2, 1>(md, xa, vec, false, s);
    case 21: return launch_x6<128, 128, 2, 4, 1>(md, xa, vec, false, s);
    case 22: return launch_x6<128, 64, 2, 2, 1>(md, xa, vec, false, s);
    case 23: return launch_x6<64, 64, 2, 2, 1>(md, xa, vec, false, s);
    case 24: return launch_x6<128, 128, 2, 2, 2>(md, xa, vec, false, s);
    case 25: return launch_x6<256, 128, 4, 2, 1>(md, xa, vec, false, s);
    case 26: return launch_x6<128, 128, 2, 4, 2>(md, xa, vec, false, s);
    case 27: return launch_x6<128, 256, 2, 4, 1>(md, xa, vec, false, s);
    case 28: return launch_x6<64, 256, 2, 4, 1>(md, xa, vec, false, s);
    default: return launch_x6<64, 128, 2, 2, 1>(md, xa, vec, false, s);
  }
}

// ---------------------------------------------------------------------------------------------
// Split-K forward (round 5): y = act(A W^T + b) at few rows (the rollout's 4096-row policy layers),
// where a row tile's whole K loop on one block leaves most CUs idle and the block's per-chunk
// latency sets the time.  k_gemm_x6 mode 4 writes S partial products (slice s: k in [s kslice,
// (s + 1) kslice)) to a workspace ws [S][M][N]; k_splitk_finish sums them in fixed order (s = 0,
// 1, ..., S - 1, then + b) and applies the ELU as epi_forward does.  Deterministic; the products
// are the exact three-term splits of k_gemm_x6, only the split-K order of the sum differs from the
// one-pass tiles.
namespace {
// SC > 0: the slice count at compile time (every slice's load issued before the first add); 0: S
template <bool ELU, int SC>
__global__ void __launch_bounds__(256) k_splitk_finish(const float* __restrict__ ws, int64_t sstride,
                                                       const float* __restrict__ bias, float* __restrict__ C,
                                                       int64_t ldc, int64_t M, int N, int S, bool vec) {
  const int nq = (N + 3) >> 2;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= M * nq) return;
  const int64_t m = t / nq;
  const int n0 = (int)(t % nq) * 4;
  const float* p = ws + m * N + n0;
  float v[4];
  if (vec) {  // N % 4 == 0, C rows 16-byte aligned
    float4 a;
    if (SC > 0) {
      typedef float fin4 __attribute__((ext_vector_type(4)));
      fin4 x[SC > 0 ? SC : 1];
#pragma unroll
      for (int s = 0; s < SC; s++) x[s] = __builtin_nontemporal_load(reinterpret_cast<const fin4*>(p + s * sstride));
#pragma unroll
      for (int s = 1; s < SC; s++) { x[0].x += x[s].x; x[0].y += x[s].y; x[0].z += x[s].z; x[0].w += x[s].w; }
      a = make_float4(x[0].x, x[0].y, x[0].z, x[0].w);
    } else {
      a = *reinterpret_cast<const float4*>(p);
      for (int s = 1; s < S; s++) {
        const float4 b = *reinterpret_cast<const float4*>(p + s * sstride);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
    }
    const float4 bb = *reinterpret_cast<const float4*>(bias + n0);
    v[0] = a.x + bb.x; v[1] = a.y + bb.y; v[2] = a.z + bb.z; v[3] = a.w + bb.w;
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (ELU) v[q] = v[q] > 0.f ? v[q] : expm1f(v[q]);
    *reinterpret_cast<float4*>(C + m * ldc + n0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int q = 0; q < 4 && n0 + q < N; q++) {
      float a = p[q];
      for (int s = 1; s < S; s++) a += p[q + s * sstride];
      float x = a + bias[n0 + q];
      if (ELU) x = x > 0.f ? x : expm1f(x);
      C[m * ldc + n0 + q] = x;
    }
  }
}

// the fixed-order sum of the slices + bias (+ ELU): one thread per 4 columns of a row
int splitk_finish(const float* ws, const float* bias, float* C, int64_t ldc, int64_t M, int N, int slices, bool elu,
                  hipStream_t s) {
  const int64_t threads = M * ((N + 3) / 4);
  const bool fvec = N % 4 == 0 && ldc % 4 == 0 && (uintptr_t)C % 16 == 0 && (uintptr_t)bias % 16 == 0;
  const dim3 grid((unsigned)((threads + 255) / 256)), block(256);
#define HG_FIN(E, SC) hipLaunchKernelGGL((k_splitk_finish<E, SC>), grid, block, 0, s, ws, M * (int64_t)N, bias, C, ldc, M, N, \
                                         slices, fvec)
  if (elu) {
    if (slices == 4) HG_FIN(true, 4);
    else if (slices == 2) HG_FIN(true, 2);
    else HG_FIN(true, 0);
  } else {
    if (slices == 4) HG_FIN(false, 4);
    else if (slices == 2) HG_FIN(false, 2);
    else HG_FIN(false, 0);
  }
#undef HG_FIN
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}
}  // namespace

extern "C" int64_t hg_gemm_splitk_kslice(int K, int slices) {
  if (K <= 0 || slices < 1) return -1;
  return (((int64_t)K + slices - 1) / slices + 15) & ~(int64_t)15;
}

extern "C" int hg_gemm_f32_splitk(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                                  float* C, int64_t ldc, float* ws, int64_t ws_floats, int64_t M, int N, int K,
                                  int act, int tile, int slices, void* stream) {
  if (!A || !B || !bias || !C || !ws || M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N ||
      act < 0 || act > 1 || tile < 20 || tile > 28 || slices < 2 || slices > 16)
    return HG_ERR_ARG;
  const int64_t kslice = hg_gemm_splitk_kslice(K, slices);
  if ((slices - 1) * kslice >= K) return HG_ERR_ARG;  // every slice holds part of the reduction
  if (ws_floats < slices * M * (int64_t)N) return HG_ERR_ARG;
  if ((uintptr_t)A % 4 || (uintptr_t)B % 4 || (uintptr_t)C % 4 || (uintptr_t)bias % 4 || (uintptr_t)ws % 16)
    return HG_ERR_ARG;
  const int64_t threads = M * ((N + 3) / 4);  // the finishing launch: one thread per 4 columns
  if ((threads + 255) / 256 > 0x7fffffff) return HG_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  GemmArgs g{A, lda, B, ldb, nullptr, nullptr, 0, ws, N, nullptr, M, N, K, 0, 0};
  GemmX6Args xa{g, kslice, M * (int64_t)N, slices};
  const bool vec = lda % 4 == 0 && ldb % 4 == 0 && (uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0;
  const bool elu = act == 1;
  const int md = 4;
  int rc;
  switch (tile) {
    case 20: rc = launch_x6<128, 128, 2, 2, 1>(md, xa, vec, elu, s); break;
    case 21: rc = launch_x6<128, 128, 2, 4, 1>(md, xa, vec, elu, s); break;
    case 22: rc = launch_x6<128, 64, 2, 2, 1>(md, xa, vec, elu, s); break;
    case 23: rc = launch_x6<64, 64, 2, 2, 1>(md, xa, vec, elu, s); break;
    case 24: rc = launch_x6<128, 128, 2, 2, 2>(md, xa, vec, elu, s); break;
    case 25: rc = launch_x6<256, 128, 4, 2, 1>(md, xa, vec, elu, s); break;
    case 26: rc = launch_x6<128, 128, 2, 4, 2>(md, xa, vec, elu, s); break;
    case 27: rc = launch_x6<128, 256, 2, 4, 1>(md, xa, vec, elu, s); break;
    default: rc = launch_x6<64, 256, 2, 4, 1>(md, xa, vec, elu, s); break;
  }
  if (rc != HG_OK) return rc;
  return splitk_finish(ws, bias, C, ldc, M, N, slices, elu, s);
}

// The same split-K forward with W as the operand image hg_gemm_x6_image_jobs builds (trans 0, N
// rows, K deep): the slices DMA B's three planes into LDS instead of splitting W per block.  The
// products and their order are those of hg_gemm_f32_splitk (bitwise the same output).  Tiles with
// one 16-deep chunk per stage only (a slice's chunks then never reach past the image's K).
extern "C" int hg_gemm_f32_splitk_img(const float* A, int64_t lda, const void* Bimg, int64_t bimg_bytes,
                                      const float* bias, float* C, int64_t ldc, float* ws, int64_t ws_floats,
                                      int64_t M, int N, int K, int act, int tile, int slices, void* stream) {
  if (!A || !Bimg || !bias || !C || !ws || M <= 0 || N <= 0 || K <= 0 || lda < K || ldc < N || act < 0 || act > 1 ||
      tile < 19 || tile > NTILES_IMG || tile == 24 || tile == 26 || tile == 29 || slices < 2 || slices > 16)
    return HG_ERR_ARG;
  if (bimg_bytes != hg_gemm_x6_image_bytes(N, K)) return HG_ERR_ARG;
  const int64_t kslice = hg_gemm_splitk_kslice(K, slices);
  if ((slices - 1) * kslice >= K) return HG_ERR_ARG;
  if (ws_floats < slices * M * (int64_t)N) return HG_ERR_ARG;
  if ((uintptr_t)A % 4 || (uintptr_t)Bimg % 16 || (uintptr_t)C % 4 || (uintptr_t)bias % 4 || (uintptr_t)ws % 16)
    return HG_ERR_ARG;
  if ((M * ((N + 3) / 4) + 255) / 256 > 0x7fffffff) return HG_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  GemmArgs g{A, lda, reinterpret_cast<const float*>(Bimg), img_rows(N) * 2, nullptr, nullptr, 0, ws, N, nullptr, M, N,
             K, 0, 0};
  GemmX6Args xa{g, kslice, M * (int64_t)N, slices};
  const bool vec = lda % 4 == 0 && (uintptr_t)A % 16 == 0;
  const int rc = x6_img_dispatch(tile, 4, 1, xa, vec, false, s);
  if (rc != HG_OK) return rc;
  return splitk_finish(ws, bias, C, ldc, M, N, slices, act == 1, s);
}

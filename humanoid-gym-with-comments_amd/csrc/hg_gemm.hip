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

  // epilogue.  acc register q of a 32x32 tile: row (q & 3) + 8 (q >> 2) + 4h, column i.
  if (MODE == 0) {
#pragma unroll
    for (int n = 0; n < TN; n++) {
      const int cidx = n0 + wn0 + 32 * n + i;
      if (cidx > nmax) continue;
      const float bc = g.bias ? g.bias[cidx] : 0.f;
#pragma unroll
      for (int m = 0; m < TM; m++) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int64_t r = m0 + wm0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
          if (r <= mmax) {
            float v = acc[m][n][q] + bc;
            if (ELU) v = v > 0.f ? v : expm1f(v);
            g.C[r * g.ldc + cidx] = v;
          }
        }
      }
    }
  } else {
    float* red = lds;  // [WGM][BN] column partials of the waves along M (staging buffers are free)
#pragma unroll
    for (int n = 0; n < TN; n++) {
      const int cl = wn0 + 32 * n + i;
      const int cidx = n0 + cl;
      float cs = 0.f;
#pragma unroll
      for (int m = 0; m < TM; m++) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int64_t r = m0 + wm0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
          float v = acc[m][n][q];
          if (r <= mmax && cidx <= nmax) {
            if (ELU) {
              const float yv = g.Y[r * g.ldY + cidx];
              v = yv > 0.f ? v : v * (yv + 1.f);
            }
            g.C[r * g.ldc + cidx] = v;
          } else {
            v = 0.f;
          }
          cs += v;
        }
      }
      cs += __shfl_xor(cs, 32);
      if (h == 0) red[(wave % WGM) * BN + cl] = cs;
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

constexpr int NTILES = 18;
// block rows of a tile id (the column-partial row count of mode 1)
int tile_bm(int tile) {
  return (tile <= 2 || (tile >= 8 && tile <= 10) || tile == 12 || tile == 13 || tile == 16 || tile == 17) ? 128 : 64;
}

}  // namespace

extern "C" int hg_gemm_tile(int mode, int64_t M, int N, int K) {
  (void)mode;
  (void)K;
  // pipelined 128 x 64 tile on 8 waves while that gives >= 3 blocks per CU, else 64 x 64
  // (scripts/gemm_probe.py, profiles/r3_gemm)
  const int64_t t16 = ((M + 127) / 128) * ((N + 63) / 64);
  return t16 >= 768 ? 16 : 5;
}

extern "C" int64_t hg_gemm_colpart_rows(int64_t M, int tile) {
  if (tile < 1 || tile > NTILES) return -1;
  const int bm = tile_bm(tile);
  return (M + bm - 1) / bm;
}

extern "C" int hg_gemm_f32(int mode, const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                           const float* Y, int64_t ldY, float* C, int64_t ldc, float* colpart, int64_t M, int N, int K,
                           int act, int tile, void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldc < N || (mode != 0 && mode != 1) || act < 0 ||
      act > 1 || tile < 1 || tile > NTILES)
    return HG_ERR_ARG;
  if (mode == 0 && ldb < K) return HG_ERR_ARG;
  if (mode == 1 && (ldb < N || (act == 1 && (!Y || ldY < N)))) return HG_ERR_ARG;
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
    default: return launch<64, 64, 2, 2, 16, 1, 1>(mode, g, vec, elu, s);
  }
}

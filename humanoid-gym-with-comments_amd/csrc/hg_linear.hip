// hg_linear.hip — fused Linear + bias + ELU forward of the policy MLPs on the f32 matrix cores
// (gfx950, v_mfma_f32_32x32x2_f32: exact f32 products, f32 accumulation).
//
// Every hidden layer of the actor / lin-vel / critic networks (actor_critic.py:36-149, nn.Linear
// followed by nn.ELU) is  y = elu(x W^T + b)  with x [rows, k] row-major (row stride ldx), W [n, k]
// row-major (nn.Linear.weight) and y [rows, n].  torch runs it as an addmm (hipBLASLt, bias in the
// GEMM epilogue) plus a separate ELU pass that reads and writes the [rows, n] output once more.
// Here the bias and the ELU are applied to the accumulators before the only store.
//
// Mapping.  x and W are both k-contiguous, so the two MFMA operands are read the same way: one
// wave owns a (32 TM) x (32 TN) output tile; lane l (i = l & 31, h = l >> 5) holds, per 32-wide
// k chunk, the 16 consecutive k values [16h, 16h + 16) of x row i of each 32-row sub-tile and of W
// row i of each 32-column sub-tile (four 16-byte loads per row, straight from global memory into
// registers — no LDS, no barriers).  MFMA step s (0..15) then takes k = 16h + s from lane half h:
// the A/B lane maps of 32x32x2 are A[i][k = h], B[k = h][j = i], so each step sums two k values
// and the 16 steps cover the chunk (a permutation of the k order inside the chunk; the sum is the
// same dot product).  The next chunk's loads are issued before the current chunk's 16 TM TN MFMAs
// (register double buffer).  MFMA per chunk per wave: 16 TM TN x 64 cycles; loads per chunk:
// 4 (TM + TN) x 1 KB through the L1 — a 2x2 tile keeps the matrix pipe the binding resource.
// Blocks of 4 waves take 4 consecutive tiles of the row-major tile grid (neighbouring waves share
// their x rows); consecutive block ids run on the same XCD (block id remapped by the 8-XCD round
// robin) so a row band's column tiles share one L2.
//
// Tails: rows / columns past the end load a clamped (valid) row and are not stored; k past the
// end loads 0 (the last, partial chunk only).  Rows not 16-byte aligned (k or ldx not a multiple
// of 4, e.g. the 705-wide actor observation) take the variant with 16-byte loads at 4-byte
// alignment and a scalar tail chunk.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hg_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));

constexpr int LIN_WAVES = 4;  // waves per block

// 16 consecutive floats p[0..16) of one operand row; k0 = first k of them, valid while k < K
template <bool VEC, bool TAIL>
__device__ __forceinline__ void ld16(const float* __restrict__ p, int k0, int K, float v[16]) {
  if (VEC && !TAIL) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const float4 t = *reinterpret_cast<const float4*>(p + 4 * q);
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
  } else if (VEC) {
    // K % 4 == 0: a 4-group is wholly in or out
#pragma unroll
    for (int q = 0; q < 4; q++) {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k0 + 4 * q < K) t = *reinterpret_cast<const float4*>(p + 4 * q);
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
  } else if (!TAIL) {
    // rows only 4-byte aligned (ldx % 4 != 0): 16-byte loads at 4-byte alignment (gfx950 global
    // loads take unaligned addresses)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const f32x4u t = *reinterpret_cast<const f32x4u*>(p + 4 * q);
      v[4 * q] = t[0]; v[4 * q + 1] = t[1]; v[4 * q + 2] = t[2]; v[4 * q + 3] = t[3];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = (k0 + j < K) ? p[j] : 0.f;
  }
}

template <int TM, int TN, bool VEC, bool TAIL>
__device__ __forceinline__ void load_chunk(const float* const* xr, const float* const* wr, int kc, int K,
                                           float a[TM][16], float w[TN][16]) {
#pragma unroll
  for (int m = 0; m < TM; m++) ld16<VEC, TAIL>(xr[m] + kc, kc, K, a[m]);
#pragma unroll
  for (int n = 0; n < TN; n++) ld16<VEC, TAIL>(wr[n] + kc, kc, K, w[n]);
}

template <int TM, int TN>
__device__ __forceinline__ void mma_chunk(const float a[TM][16], const float w[TN][16], f32x16 acc[TM][TN]) {
#pragma unroll
  for (int s = 0; s < 16; s++)
#pragma unroll
    for (int m = 0; m < TM; m++)
#pragma unroll
      for (int n = 0; n < TN; n++) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m][s], w[n][s], acc[m][n], 0, 0, 0);
}

// VEC: x and W rows 16-byte aligned (k % 4 == 0); otherwise 16-byte loads at 4-byte alignment and a
// scalar tail.
template <int TM, int TN, int S, bool VEC, bool ELU>
__global__ void __launch_bounds__(64 * LIN_WAVES) k_linear_act(const float* __restrict__ x, int64_t ldx,
                                                               const float* __restrict__ W,
                                                               const float* __restrict__ b, float* __restrict__ y,
                                                               int64_t ldy, int64_t rows, int N, int K,
                                                               int tiles_n, int64_t tiles) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 31, h = lane >> 5;
  // XCD-aware block order: hardware block id b runs on XCD b % 8; logical block L = consecutive
  // ids per XCD, so neighbouring tiles (same row band) share that XCD's L2
  const unsigned nb = gridDim.x;
  unsigned L = blockIdx.x;
  if ((nb & 7u) == 0) L = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
  const int64_t t = (int64_t)L * LIN_WAVES + (threadIdx.x >> 6);
  if (t >= tiles) return;  // whole wave exits: no barriers in this kernel
  const int64_t r0 = (t / tiles_n) * (32 * TM);
  const int c0 = (int)(t % tiles_n) * (32 * TN);

  const float* xr[TM];
  const float* wr[TN];
#pragma unroll
  for (int m = 0; m < TM; m++) {
    const int64_t r = min<int64_t>(r0 + 32 * m + i, rows - 1);
    xr[m] = x + r * ldx + 16 * h;
  }
#pragma unroll
  for (int n = 0; n < TN; n++) {
    const int c = min(c0 + 32 * n + i, N - 1);
    wr[n] = W + (int64_t)c * K + 16 * h;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; m++)
#pragma unroll
    for (int n = 0; n < TN; n++) acc[m][n] = (f32x16)0.f;

  const int kfull = K & ~31;  // chunks with all 32 k in range
  // S-stage register pipeline over the full chunks: chunk c's loads are issued S - 1 chunks ahead
  // of its MFMAs (buffer indices are compile-time: the stage loop is fully unrolled).  S = 2: three
  // and four stages measured no faster (scripts/linear_probe.py), the register cost drops occupancy
  float a[S][TM][16], w[S][TN][16];
#pragma unroll
  for (int j = 0; j < S - 1; j++)
    if (32 * j < kfull) load_chunk<TM, TN, VEC, false>(xr, wr, 32 * j, K, a[j], w[j]);
  for (int kb = 0; kb < kfull; kb += 32 * S) {
#pragma unroll
    for (int j = 0; j < S; j++) {
      const int kn = kb + 32 * (j + S - 1);
      if (kn < kfull) load_chunk<TM, TN, VEC, false>(xr, wr, kn, K, a[(j + S - 1) % S], w[(j + S - 1) % S]);
      if (kb + 32 * j < kfull) mma_chunk<TM, TN>(a[j], w[j], acc);
    }
  }
  const int kc = kfull;
  if (kc < K) {  // partial chunk: k = kc + 16h + j valid while < K
    load_chunk<TM, TN, VEC, true>(xr, wr, kc, K - 16 * h, a[0], w[0]);
    mma_chunk<TM, TN>(a[0], w[0], acc);
  }

  // epilogue: + bias, ELU, one store.  acc register q of a 32x32 tile: row (q & 3) + 8 (q >> 2)
  // + 4h, column i.  The bias is read once per column, unconditionally (clamped column) and
  // retired before the stores (round 5): read inside the column guard, the compiler waited vmcnt(0)
  // for it in front of every store, and stores count on that counter — 16-64 serialized stores
#pragma unroll
  for (int n = 0; n < TN; n++) {
    const int c = c0 + 32 * n + i;
    float bc = b ? b[min(c, N - 1)] : 0.f;
    asm volatile("" : "+v"(bc));
    if (c >= N) continue;
#pragma unroll
    for (int m = 0; m < TM; m++) {
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const int64_t r = r0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (r < rows) {
          float v = acc[m][n][q] + bc;
          if (ELU) v = v > 0.f ? v : expm1f(v);
          y[r * ldy + c] = v;
        }
      }
    }
  }
}

// Small-output variant: one wave per 16 x 16 tile (hg_lin16_acc, hg_common.h: shared with the
// rollout's fused policy tail in hg_rollout.hip, so the two give the same bits).  Four times the
// waves of the 32 x 32 tile for the same output, for the latency-bound 4096-row rollout layers.
template <bool VEC, bool ELU>
__global__ void __launch_bounds__(64 * LIN_WAVES) k_linear_act16(const float* __restrict__ x, int64_t ldx,
                                                                 const float* __restrict__ W,
                                                                 const float* __restrict__ b, float* __restrict__ y,
                                                                 int64_t ldy, int64_t rows, int N, int K,
                                                                 int tiles_n, int64_t tiles) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const unsigned nb = gridDim.x;
  unsigned L = blockIdx.x;
  if ((nb & 7u) == 0) L = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
  const int64_t t = (int64_t)L * LIN_WAVES + (threadIdx.x >> 6);
  if (t >= tiles) return;
  const int64_t r0 = (t / tiles_n) * 16;
  const int c0 = (int)(t % tiles_n) * 16;
  const float* xr = x + min<int64_t>(r0 + i, rows - 1) * ldx + 8 * g;
  const float* wr = W + (int64_t)min(c0 + i, N - 1) * K + 8 * g;
  hg_f32x4 acc0, acc1;
  hg_lin16_acc<VEC>(xr, wr, K, g, acc0, acc1);
  const int c = c0 + i;
  if (c >= N) return;
  const float bc = b ? b[c] : 0.f;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int64_t r = r0 + 4 * g + q;
    if (r < rows) {
      float v = acc0[q] + acc1[q] + bc;
      if (ELU) v = v > 0.f ? v : expm1f(v);
      y[r * ldy + c] = v;
    }
  }
}

int launch_linear16(const float* x, int64_t ldx, const float* W, const float* b, float* y, int64_t ldy, int64_t rows,
                    int n, int k, bool vec, bool elu, hipStream_t s) {
  const int tiles_n = (n + 15) / 16;
  const int64_t tiles = ((rows + 15) / 16) * tiles_n;
  const int64_t blocks = (tiles + LIN_WAVES - 1) / LIN_WAVES;
  if (blocks > 0x7fffffff) return HG_ERR_ARG;
  const dim3 grid((unsigned)blocks), block(64 * LIN_WAVES);
#define HG_LIN16(V, E) \
  hipLaunchKernelGGL((k_linear_act16<V, E>), grid, block, 0, s, x, ldx, W, b, y, ldy, rows, n, k, tiles_n, tiles)
  if (vec && elu) HG_LIN16(true, true);
  else if (vec) HG_LIN16(true, false);
  else if (elu) HG_LIN16(false, true);
  else HG_LIN16(false, false);
#undef HG_LIN16
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

template <int TM, int TN, int S>
int launch_linear(const float* x, int64_t ldx, const float* W, const float* b, float* y, int64_t ldy, int64_t rows,
                  int n, int k, bool vec, bool elu, hipStream_t s) {
  const int tiles_n = (n + 32 * TN - 1) / (32 * TN);
  const int64_t tiles = ((rows + 32 * TM - 1) / (32 * TM)) * tiles_n;
  const int64_t blocks = (tiles + LIN_WAVES - 1) / LIN_WAVES;
  if (blocks > 0x7fffffff) return HG_ERR_ARG;
  const dim3 grid((unsigned)blocks), block(64 * LIN_WAVES);
#define HG_LIN(V, E) \
  hipLaunchKernelGGL((k_linear_act<TM, TN, S, V, E>), grid, block, 0, s, x, ldx, W, b, y, ldy, rows, n, k, tiles_n, tiles)
  if (vec && elu) HG_LIN(true, true);
  else if (vec) HG_LIN(true, false);
  else if (elu) HG_LIN(false, true);
  else HG_LIN(false, false);
#undef HG_LIN
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

}  // namespace

// Wave-tile choice (scripts/linear_probe.py on MI355X over the policy MLPs' shapes,
// profiles/r2_v3/linear_probe*.jsonl): 64 x 32 while that still gives >= 2048 waves (2 per SIMD);
// below one 32 x 32 wave per SIMD the 16 x 16 tile (4x the waves: 4096-row 256 -> 128 layer
// 13.8 -> 10.6 us, 128 -> 128 10.5 -> 7.6 us); 32 x 32 otherwise.  tile 1..5 forces 64x64, 64x32,
// 32x64, 32x32, 16x16.
extern "C" int hg_linear_act_tile(int64_t rows, int n, int k) {
  (void)k;
  const int64_t waves21 = ((rows + 63) / 64) * ((n + 31) / 32);
  const int64_t waves11 = ((rows + 31) / 32) * ((n + 31) / 32);
  return waves21 >= 2048 ? 2 : (waves11 < 1024 ? 5 : 4);
}

extern "C" int hg_linear_act_forward(const float* x, int64_t ldx, const float* W, const float* b, float* y,
                                     int64_t ldy, int64_t rows, int n, int k, int act, int tile, void* stream) {
  if (!x || !W || !y || rows <= 0 || n <= 0 || k <= 0 || ldx < k || ldy < n || (act != 0 && act != 1) || tile < 0 ||
      tile > 5)
    return HG_ERR_ARG;
  if ((uintptr_t)x % 4 != 0 || (uintptr_t)W % 4 != 0) return HG_ERR_ARG;
  const bool vec = ldx % 4 == 0 && k % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)W % 16 == 0;
  const bool elu = act == 1;
  if (tile == 0) tile = hg_linear_act_tile(rows, n, k);
  hipStream_t s = (hipStream_t)stream;
  switch (tile) {
    case 1: return launch_linear<2, 2, 2>(x, ldx, W, b, y, ldy, rows, n, k, vec, elu, s);
    case 2: return launch_linear<2, 1, 2>(x, ldx, W, b, y, ldy, rows, n, k, vec, elu, s);
    case 3: return launch_linear<1, 2, 2>(x, ldx, W, b, y, ldy, rows, n, k, vec, elu, s);
    case 4: return launch_linear<1, 1, 2>(x, ldx, W, b, y, ldy, rows, n, k, vec, elu, s);
    default: return launch_linear16(x, ldx, W, b, y, ldy, rows, n, k, vec, elu, s);
  }
}

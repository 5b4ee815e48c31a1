// hg_policy.hip — the rollout's policy forward as ONE kernel (gfx950).
//
// Replaces, on the device rollout (PPO.act -> ActorCritic.actor, actor_critic.py:36-149 of the
// reference), the actor MLP's four launches — hidden layers K0 -> N1 -> N2 -> N3 with bias + ELU,
// then the skinny N3 -> nout output layer (705 -> 512 -> 256 -> 128 -> 12 for XBot-L) — by one
// launch whose activations never leave the CU: a block owns 32 rows of the batch and runs the
// whole chain, the hidden activations in LDS (f32).
//
// Arithmetic: every hidden product is the f32 product on the bf16 matrix cores as in hg_gemm.hip's
// bf16-split kernels — both operands split exactly into three bf16 terms, the six products of
// total order <= 2 accumulated in f32 by v_mfma_f32_32x32x16_bf16, smallest terms first (error per
// element below torch's f32 GEMM's, tests/test_gpu_gemm.py) — with the weights read from the
// operand images hg_gemm_x6_image_jobs builds (trans 0, W [N, K] row-major); the output layer is
// f32 FMAs in k order.  Mapping: block = 4 waves, 32 rows; layer l's N_l columns split over the 4
// waves (each a 32-row x N_l / 4 strip of 32x32 accumulators); the A fragments (row i, 8
// consecutive k) come straight from the input rows (layer 0, global) or the LDS activations and are
// split in registers; the B fragments come from the image in L2 straight into registers, one
// 16-deep chunk ahead of the MFMAs.  No barrier inside a layer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hg_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int ROWS = 32;   // batch rows per block
constexpr int NW = 4;      // waves per block
constexpr int NT = 64 * NW;
constexpr int PAD = 4;     // LDS row padding (floats): conflict-free 16-byte fragment reads
constexpr int MAX_OUT = 16;

// x = x0 + x1 + x2 exactly (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)), as hg_gemm.hip
__device__ __forceinline__ void split3(const float v[8], bf16x8& x0, bf16x8& x1, bf16x8& x2) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const __bf16 a = (__bf16)v[j];
    const float r1 = v[j] - (float)a;
    const __bf16 b = (__bf16)r1;
    const float r2 = r1 - (float)b;
    x0[j] = a;
    x1[j] = b;
    x2[j] = (__bf16)r2;
  }
}

// image slots per plane of an R-row operand (hg_gemm_x6_image_jobs: rows padded to 256, 16-byte slots)
__host__ __device__ inline int64_t img_pitch(int64_t R) { return (R + 255) / 256 * 256 * 2; }

// One hidden layer: Hout[32][N] (LDS, row stride N + PAD) = elu(A[32][K] W^T + b).  A: global rows
// (layer 0; rows past rmax read row rmax, k past K read 0) or LDS (row stride lda, K a multiple of
// 16).  img: W's image (pitch slots per plane).
template <int N, bool GLOBAL>
__device__ __forceinline__ void hidden_layer(const float* __restrict__ A, int64_t lda, int rmax, int K,
                                             const bf16x8* __restrict__ img, const float* __restrict__ bias,
                                             float* __restrict__ Hout, int wave, int lane) {
  constexpr int TN = N / NW / 32;
  static_assert(TN >= 1 && N == NW * 32 * TN, "columns per wave");
  const int i = lane & 31, h = lane >> 5;
  const int nw0 = wave * (N / NW);
  const int64_t pitch = img_pitch(N);
  const bf16x8* bbase = img + ((nw0 >> 5) * 2 + h) * 32 + i;
  const float* arow = A + (int64_t)(GLOBAL ? min(i, rmax) : i) * lda;
  const int nchunks = (K + 15) / 16;
  f32x16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; t++) acc[t] = (f32x16)0.f;

  auto loadA = [&](int c, float v[8]) {
    const int k0 = 16 * c + 8 * h;
    const float* p = arow + k0;
    if (!GLOBAL) {  // LDS rows: 16-byte aligned (row stride (N + PAD) * 4 bytes, k0 a multiple of 8)
      const float4 x = *reinterpret_cast<const float4*>(p), y = *reinterpret_cast<const float4*>(p + 4);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    } else if (k0 + 8 <= K) {  // input rows: 4-byte aligned (a strided view of the history window)
      const f32x4u x = *reinterpret_cast<const f32x4u*>(p), y = *reinterpret_cast<const f32x4u*>(p + 4);
#pragma unroll
      for (int q = 0; q < 4; q++) { v[q] = x[q]; v[4 + q] = y[q]; }
    } else {
#pragma unroll
      for (int q = 0; q < 8; q++) v[q] = (k0 + q < K) ? p[q] : 0.f;
    }
  };
  auto loadB = [&](int c, bf16x8 b[3][TN]) {
#pragma unroll
    for (int p = 0; p < 3; p++)
#pragma unroll
      for (int t = 0; t < TN; t++) b[p][t] = bbase[((int64_t)c * 3 + p) * pitch + t * 64];
  };
  float va[8];
  bf16x8 bc[3][TN];
  loadA(0, va);
  loadB(0, bc);
  for (int c = 0; c < nchunks; c++) {
    float vn[8];
    bf16x8 bn[3][TN];
    const bool more = c + 1 < nchunks;
    if (more) {
      loadA(c + 1, vn);
      loadB(c + 1, bn);
    }
    bf16x8 a0, a1, a2;
    split3(va, a0, a1, a2);
#pragma unroll
    for (int t = 0; t < TN; t++) {
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, bc[0][t], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bc[1][t], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bc[2][t], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bc[0][t], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bc[1][t], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bc[0][t], acc[t], 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int q = 0; q < 8; q++) va[q] = vn[q];
#pragma unroll
      for (int p = 0; p < 3; p++)
#pragma unroll
        for (int t = 0; t < TN; t++) bc[p][t] = bn[p][t];
    }
  }
  // accumulator register q of a 32x32 tile: row (q & 3) + 8 (q >> 2) + 4h, column i
#pragma unroll
  for (int t = 0; t < TN; t++) {
    const int col = nw0 + 32 * t + i;
    const float bcol = bias[col];
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int r = (q & 3) + 8 * (q >> 2) + 4 * h;
      float v = acc[t][q] + bcol;
      v = v > 0.f ? v : expm1f(v);
      Hout[r * (N + PAD) + col] = v;
    }
  }
}

template <int N1, int N2, int N3>
__global__ void __launch_bounds__(NT) k_policy_x6(const float* __restrict__ x, int64_t ldx, int64_t rows, int K0,
                                                  const bf16x8* __restrict__ img1, const bf16x8* __restrict__ img2,
                                                  const bf16x8* __restrict__ img3, const float* __restrict__ b1,
                                                  const float* __restrict__ b2, const float* __restrict__ b3,
                                                  const float* __restrict__ Wl, const float* __restrict__ bl, int nout,
                                                  float* __restrict__ y, int64_t ldy) {
  constexpr int S1 = ROWS * (N1 + PAD), S2 = ROWS * (N2 + PAD), S3 = ROWS * (N3 + PAD);
  static_assert(S3 <= S1, "layer 3 reuses layer 1's buffer");
  __shared__ __attribute__((aligned(16))) float H1[S1];   // layer 1 output, then layer 3's
  __shared__ __attribute__((aligned(16))) float H2[S2];
  __shared__ __attribute__((aligned(16))) float WL[MAX_OUT * (N3 + PAD)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int rvalid = (int)min<int64_t>(ROWS, rows - r0);
  // the output layer's weights, staged once
  for (int e = tid; e < nout * N3; e += NT) WL[(e / N3) * (N3 + PAD) + e % N3] = Wl[e];
  hidden_layer<N1, true>(x + r0 * ldx, ldx, rvalid - 1, K0, img1, b1, H1, wave, lane);
  __syncthreads();
  hidden_layer<N2, false>(H1, N1 + PAD, ROWS - 1, N1, img2, b2, H2, wave, lane);
  __syncthreads();  // every wave is done reading H1 before layer 3 overwrites it
  hidden_layer<N3, false>(H2, N2 + PAD, ROWS - 1, N2, img3, b3, H1, wave, lane);
  __syncthreads();
  // output layer: thread (row r, outputs j and j + 8), f32 FMAs in k order, 4 k per step
  const int r = tid >> 3, j0 = tid & 7;
  const float* hr = H1 + r * (N3 + PAD);
#pragma unroll
  for (int half = 0; half < 2; half++) {
    const int j = j0 + 8 * half;
    if (j >= nout) break;
    const float* w = WL + j * (N3 + PAD);
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < N3; k += 4) {
      const float4 hv = *reinterpret_cast<const float4*>(hr + k);
      const float4 wv = *reinterpret_cast<const float4*>(w + k);
      s = fmaf(hv.x, wv.x, s);
      s = fmaf(hv.y, wv.y, s);
      s = fmaf(hv.z, wv.z, s);
      s = fmaf(hv.w, wv.w, s);
    }
    if (r < rvalid) y[(r0 + r) * ldy + j] = s + bl[j];
  }
}

}  // namespace

extern "C" int hg_policy_forward(const float* x, int64_t ldx, int64_t rows, int K0, int n1, int n2, int n3,
                                 const void* const* images, const int64_t* image_bytes, const float* const* biases,
                                 const float* Wl, const float* bl, int nout, float* y, int64_t ldy, void* stream) {
  if (!x || !images || !image_bytes || !biases || !Wl || !bl || !y || rows <= 0 || K0 <= 0 || K0 > 0x3fffffff ||
      ldx < K0 || nout <= 0 || nout > MAX_OUT || ldy < nout)
    return HG_ERR_ARG;
  if (n1 != 512 || n2 != 256 || n3 != 128) return HG_ERR_ARG;  // the instantiated chain (XBot-L actor)
  const int64_t want[3] = {hg_gemm_x6_image_bytes(n1, K0), hg_gemm_x6_image_bytes(n2, n1),
                           hg_gemm_x6_image_bytes(n3, n2)};
  for (int l = 0; l < 3; l++)
    if (!images[l] || !biases[l] || image_bytes[l] != want[l] || (uintptr_t)images[l] % 16) return HG_ERR_ARG;
  if ((uintptr_t)x % 4 || (uintptr_t)y % 4 || (uintptr_t)Wl % 4) return HG_ERR_ARG;
  const int64_t blocks = (rows + ROWS - 1) / ROWS;
  if (blocks > 0x7fffffff) return HG_ERR_ARG;
  hipLaunchKernelGGL((k_policy_x6<512, 256, 128>), dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, x, ldx,
                     rows, K0, reinterpret_cast<const bf16x8*>(images[0]), reinterpret_cast<const bf16x8*>(images[1]),
                     reinterpret_cast<const bf16x8*>(images[2]), biases[0], biases[1], biases[2], Wl, bl, nout, y,
                     ldy);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

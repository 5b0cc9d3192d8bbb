// PointNetfeat forward on gfx950 (models/pointnet.py:109-132).
//
// k_point_mlp3  : relu(conv1) -> relu(conv2) -> relu(conv3) for a 64-point tile
//                 of one cloud.  conv1 (K=3) on the VALU, conv2/conv3 (K=64) on
//                 the f32 MFMA (v_mfma_f32_32x32x2_f32, exact f32).  Saves x1,
//                 x2, x3 point-major for the backward.
// k_conv_max128 : conv4 (128 -> O) + max/argmax over all points.  Weights are
//                 stationary in VGPRs (one 32-channel slice per wave), point
//                 tiles stream through a double-buffered LDS ring, the max is
//                 reduced in the MFMA epilogue, so the B x 1024 x N conv4 output
//                 is never materialised.
#include "common.h"

namespace pcadv {

constexpr int MLP_TILE = 64;

__global__ void __launch_bounds__(256)
k_point_mlp3(const float* __restrict__ pts_a, const float* __restrict__ pts_b, int split, int N,
             const float* __restrict__ w1, const float* __restrict__ b1,
             const float* __restrict__ w2, const float* __restrict__ b2,
             const float* __restrict__ w3, const float* __restrict__ b3,
             float* __restrict__ x1, float* __restrict__ x2, float* __restrict__ x3,
             int32_t* inc_counter) {
  __shared__ __attribute__((aligned(16))) float lds[MLP_TILE * 4 + 2 * MLP_TILE * S64];
  float* p_s = lds;                         // [64][4]
  float* x1_s = lds + MLP_TILE * 4;         // [64][68]
  float* x2_s = x1_s + MLP_TILE * S64;      // [64][68]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y, p0 = blockIdx.x * MLP_TILE;
  if (inc_counter && tid == 0 && c == 0 && blockIdx.x == 0) *inc_counter += 1;
  const float* pts = c < split ? pts_a + (size_t)c * N * 3 : pts_b + (size_t)(c - split) * N * 3;

  if (tid < MLP_TILE * 3) {
    const int p = tid / 3, k = tid % 3;
    p_s[p * 4 + k] = (p0 + p < N) ? pts[(size_t)(p0 + p) * 3 + k] : 0.f;
  }
  __syncthreads();

  // conv1 (3 -> 64) + relu on the VALU: thread = (channel, 16-point group)
  {
    const int ch = tid & 63, pg = tid >> 6;
    const float wa = w1[ch * 3 + 0], wb = w1[ch * 3 + 1], wc = w1[ch * 3 + 2], bb = b1[ch];
    const size_t gbase = ((size_t)c * N + p0) * 64;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int p = pg * 16 + i;
      float v = fmaf(wc, p_s[p * 4 + 2], fmaf(wb, p_s[p * 4 + 1], fmaf(wa, p_s[p * 4 + 0], bb)));
      v = v > 0.f ? v : 0.f;
      if (p0 + p >= N) v = 0.f;
      x1_s[p * S64 + ch] = v;
      if (p0 + p < N) x1[gbase + (size_t)p * 64 + ch] = v;
    }
  }
  __syncthreads();

  // conv2 (64 -> 64) + relu on MFMA: wave -> (point tile, channel tile)
  {
    const int pt = wave >> 1, ct = wave & 1;
    f32x4 bf[8];
    load_bfrag<64>(w2, 32 * ct, lane, bf);
    f32x16 acc = {};
    acc = mfma_rows_x_wt<64>(x1_s + 32 * pt * S64, S64, bf, acc, lane);
    const int col = 32 * ct + (lane & 31);
    const float bias = b2[col];
    const size_t gbase = ((size_t)c * N + p0) * 64;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * pt + acc_row(r, lane);
      float v = acc[r] + bias;
      v = v > 0.f ? v : 0.f;
      x2_s[row * S64 + col] = v;
      if (p0 + row < N) x2[gbase + (size_t)row * 64 + col] = v;
    }
  }
  __syncthreads();

  // conv3 (64 -> 128) + relu on MFMA: wave -> 32-channel slice, both point tiles
  {
    f32x4 bf[8];
    load_bfrag<64>(w3, 32 * wave, lane, bf);
    f32x16 acc0 = {}, acc1 = {};
    acc0 = mfma_rows_x_wt<64>(x2_s, S64, bf, acc0, lane);
    acc1 = mfma_rows_x_wt<64>(x2_s + 32 * S64, S64, bf, acc1, lane);
    const int col = 32 * wave + (lane & 31);
    const float bias = b3[col];
    const size_t gbase = ((size_t)c * N + p0) * 128;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = acc_row(r, lane);
      float v0 = acc0[r] + bias, v1 = acc1[r] + bias;
      v0 = v0 > 0.f ? v0 : 0.f;
      v1 = v1 > 0.f ? v1 : 0.f;
      if (p0 + row < N) x3[gbase + (size_t)row * 128 + col] = v0;
      if (p0 + 32 + row < N) x3[gbase + (size_t)(32 + row) * 128 + col] = v1;
    }
  }
}

constexpr int CM_TILE = 64;  // points per LDS tile

template <bool RELU>
__global__ void __launch_bounds__(256, 2)
k_conv_max128(const float* __restrict__ x, int N, const float* __restrict__ w,
              const float* __restrict__ b, int O, float* __restrict__ gmax,
              int32_t* __restrict__ gidx) {
  __shared__ __attribute__((aligned(16))) float xs[2][CM_TILE * S128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y;
  const int o0 = blockIdx.x * 128 + wave * 32;
  const float* xc = x + (size_t)c * N * 128;

  f32x4 bf[16];
  load_bfrag<128>(w, o0, lane, bf);
  const float bias = b[o0 + (lane & 31)];

  // staging: 64 rows x 32 float4 = 2048 float4 per tile, 8 per thread
  f32x4 stg[8];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = tid + 256 * i, row = q >> 5, c4 = q & 31;
      stg[i] = (t0 + row < N) ? *reinterpret_cast<const f32x4*>(xc + (size_t)(t0 + row) * 128 + 4 * c4)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = tid + 256 * i, row = q >> 5, c4 = q & 31;
      *reinterpret_cast<f32x4*>(&xs[buf][row * S128 + 4 * c4]) = stg[i];
    }
  };

  float best = -INFINITY;
  int bidx = 0;
  const int ntiles = (N + CM_TILE - 1) / CM_TILE;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) gload((t + 1) * CM_TILE);
    f32x16 acc0 = {}, acc1 = {};
    {
      const int r = lane & 31, h = lane >> 5;
      const float* a0p = &xs[buf][r * S128 + 4 * h];
      const float* a1p = a0p + 32 * S128;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(a0p + 8 * g);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(a1p + 8 * g);
        acc0 = mfma32(a0.x, bf[g].x, acc0);
        acc1 = mfma32(a1.x, bf[g].x, acc1);
        acc0 = mfma32(a0.y, bf[g].y, acc0);
        acc1 = mfma32(a1.y, bf[g].y, acc1);
        acc0 = mfma32(a0.z, bf[g].z, acc0);
        acc1 = mfma32(a1.z, bf[g].z, acc1);
        acc0 = mfma32(a0.w, bf[g].w, acc0);
        acc1 = mfma32(a1.w, bf[g].w, acc1);
      }
    }
    const int base = t * CM_TILE;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = base + acc_row(r, lane);
      float v = acc0[r] + bias;
      if (RELU) v = v > 0.f ? v : 0.f;
      if (p < N && beats(v, best)) { best = v; bidx = p; }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = base + 32 + acc_row(r, lane);
      float v = acc1[r] + bias;
      if (RELU) v = v > 0.f ? v : 0.f;
      if (p < N && beats(v, best)) { best = v; bidx = p; }
    }
    if (t + 1 < ntiles) lstore(buf ^ 1);
    __syncthreads();
  }
  // lanes l and l+32 hold the same channel over interleaved rows
  const float ob = __shfl_xor(best, 32);
  const int oi = __shfl_xor(bidx, 32);
  if (beats(ob, best) || (ob == best && oi < bidx) || (ob != ob && best != best && oi < bidx)) {
    best = ob;
    bidx = oi;
  }
  if (lane < 32) {
    gmax[(size_t)c * O + o0 + lane] = best;
    gidx[(size_t)c * O + o0 + lane] = bidx;
  }
}

int launch_point_mlp3(const float* pts_a, const float* pts_b, int split, int C, int N,
                      const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* w3, const float* b3, float* x1, float* x2, float* x3,
                      int32_t* inc_counter, hipStream_t s) {
  dim3 grid((N + MLP_TILE - 1) / MLP_TILE, C);
  hipLaunchKernelGGL(k_point_mlp3, grid, dim3(256), 0, s, pts_a, pts_b, split, N, w1, b1, w2,
                     b2, w3, b3, x1, x2, x3, inc_counter);
  PC_HIP_CHECK_LAUNCH("k_point_mlp3");
  return PCADV_OK;
}

int launch_conv4_max(const float*, int, int, const float*, const float*, float*, int32_t*,
                     hipStream_t, int, int relu = 0);

int launch_conv_max128(const float* x, int C, int N, const float* w, const float* b, int O,
                       bool relu, float* gmax, int32_t* gidx, hipStream_t s) {
  if (O == PCADV_C4) {
    // the 1024-channel layers (feature conv4, the T-Nets' conv3) on the fused
    // forward's k_conv4_max: split-product screening + exact f32 re-evaluation
    // of every winner, ~4x this file's f32 kernel
    // (the ReLU before the max applied in its epilogue)
    return launch_conv4_max(x, C, N, w, b, gmax, gidx, s, 0, relu ? 1 : 0);
  }
  dim3 grid(O / 128, C);
  if (relu)
    hipLaunchKernelGGL(k_conv_max128<true>, grid, dim3(256), 0, s, x, N, w, b, O, gmax, gidx);
  else
    hipLaunchKernelGGL(k_conv_max128<false>, grid, dim3(256), 0, s, x, N, w, b, O, gmax, gidx);
  PC_HIP_CHECK_LAUNCH("k_conv_max128");
  return PCADV_OK;
}

}  // namespace pcadv

// Point-wise layers of the feature-transform path on gfx950
// (PointNetCls(feature_transform=True): STNkd models/pointnet.py:46-79, the
// feature transform bmm :118-122, feature_transform_regularizer :345-353).
//
//   k_pw_fwd        y = act(x w^T + b) over rows = points (1x1 Conv1d), K = 64/128
//                   on v_mfma_f32_32x32x2_f32; K = 3 on the VALU.  The weight may
//                   be one matrix per cloud in either layout, so the same kernel
//                   runs the per-cloud transform x2 . T (bmm).
//   k_pw_bwd_data   dx = (dy * act'(y)) w, optionally accumulated into dx
//   k_pw_bwd_weight per-256-row partial dW / db slabs (one group = all rows, or
//                   one cloud for dT), then k_pw_reduce sums the slabs in order
//   k_convmax_bwd   sparse backward of conv + max over points (optionally with
//                   the ReLU before the max): dW/db by gathering the argmax rows,
//                   dX rows from the hits sorted by channel (deterministic)
//   k_tnet_reg      ||T T^T - I||_F per cloud, and its gradient
// All reductions run in a fixed order: results are bitwise reproducible.
#include "common.h"

namespace pcadv {

constexpr int PW_ROWS = 64;   // points per workgroup tile
constexpr int PW_T = 256;     // 4 waves
constexpr int PWW_ROWS = 128; // rows per weight-gradient slab (M / 128 workgroups: 256 at 32 clouds x 1024 points)
constexpr int PWW_SUB = 32;   // rows staged in LDS at a time by the weight kernel

// A weight operand: conv layout W[o][k], or "kmajor" T[k][o] (the bmm's
// transform); one matrix per `rows_per_w` rows when rows_per_w > 0.
struct WView {
  const float* w;
  int O, K;
  int kmajor;
  int rows_per_w;
  long long stride;
  __device__ const float* base(int row0) const {
    return rows_per_w ? w + (size_t)(row0 / rows_per_w) * stride : w;
  }
  __device__ float get(const float* b, int o, int k) const {
    return kmajor ? b[(size_t)k * O + o] : b[(size_t)o * K + k];
  }
  // 16-B loads of four contiguous weights need every matrix 16-B aligned: the
  // base and, with one matrix per rows_per_w rows, the per-matrix stride (O, K
  // and the fragment offsets are multiples of 4 here)
  __device__ bool aligned16() const {
    return (reinterpret_cast<uintptr_t>(w) & 15) == 0 && (rows_per_w == 0 || (stride & 3) == 0);
  }
};

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int K, int ACT>
__global__ void __launch_bounds__(PW_T)
k_pw_fwd(const float* __restrict__ x, int M, WView wv, const float* __restrict__ b,
         float* __restrict__ y) {
  constexpr int SK = K + 4;
  __shared__ __attribute__((aligned(16))) float xs[PW_ROWS * SK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * PW_ROWS, o0 = blockIdx.y * 128;
  const int O = wv.O;
  const float* w = wv.base(r0);
  // wave -> (32-column tile, 32-row tiles): four column tiles over both row
  // tiles, or with O - o0 = 64 two column tiles x one row tile each, so every
  // wave works
  const bool narrow = O - o0 <= 64;
  const int oc = o0 + 32 * (narrow ? (wave & 1) : wave);
  const int rt0 = narrow ? (wave >> 1) : 0, nrt = narrow ? 1 : 2;
  const bool on = oc < O;  // O % 32 == 0: whole waves
  const int r = lane & 31, h = lane >> 5;
  // the weight fragments issued first: in flight during the x staging
  f32x4 bf[K / 8];
  if (on) {
    if (!wv.kmajor && wv.aligned16()) {  // (o, k..k+3) contiguous: one 16-B load each
#pragma unroll
      for (int g = 0; g < K / 8; ++g)
        bf[g] = *reinterpret_cast<const f32x4*>(w + (size_t)(oc + r) * K + 8 * g + 4 * h);
    } else {
#pragma unroll
      for (int g = 0; g < K / 8; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[g][j] = wv.get(w, oc + r, 8 * g + 4 * h + j);
    }
  }
  const int col = oc + r;
  const float bias = (b && on) ? b[col] : 0.f;
  for (int e = tid; e < PW_ROWS * K / 4; e += PW_T) {
    const int row = e / (K / 4), c4 = e % (K / 4);
    const f32x4 v = r0 + row < M ? *reinterpret_cast<const f32x4*>(x + (size_t)(r0 + row) * K + 4 * c4)
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(xs + row * SK + 4 * c4) = v;
  }
  __syncthreads();
  if (!on) return;
  for (int t = rt0; t < rt0 + nrt; ++t) {
    f32x16 acc = {};
    acc = mfma_rows_x_wt<K>(xs + 32 * t * SK, SK, bf, acc, lane);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ra = r0 + 32 * t + acc_row(i, lane);
      if (ra < M) y[(size_t)ra * O + col] = act_fwd(acc[i] + bias, ACT);
    }
  }
}

// K = 3 (conv1 on the points): thread = (column, 32-row group), VALU, the fma
// order of conv1_point (shared with the fused classifier kernels)
template <int ACT>
__global__ void __launch_bounds__(PW_T)
k_pw_fwd3(const float* __restrict__ x, int M, WView wv, const float* __restrict__ b,
          float* __restrict__ y) {
  __shared__ float xs[PW_ROWS * 4];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * PW_ROWS, o0 = blockIdx.y * 128;
  const int O = wv.O;
  const float* w = wv.base(r0);
  if (tid < PW_ROWS * 3) {
    const int row = tid / 3, k = tid % 3;
    xs[row * 4 + k] = r0 + row < M ? x[(size_t)(r0 + row) * 3 + k] : 0.f;
  }
  __syncthreads();
  const int o = o0 + (tid & 127), rg = tid >> 7;
  if (o >= O) return;
  const float wa = wv.get(w, o, 0), wb = wv.get(w, o, 1), wc = wv.get(w, o, 2);
  const float bb = b ? b[o] : 0.f;
  for (int i = 0; i < 32; ++i) {
    const int row = 32 * rg + i;
    if (r0 + row >= M) break;
    const float v = fmaf(wc, xs[row * 4 + 2], fmaf(wb, xs[row * 4 + 1], fmaf(wa, xs[row * 4], bb)));
    y[(size_t)(r0 + row) * O + o] = act_fwd(v, ACT);
  }
}

// ---------------------------------------------------------------------------
// forward chains: consecutive point-wise layers of a 64-row tile in ONE launch
// (the feature-transform extractor's conv1 -> conv2 -> STNkd conv1 -> STNkd
// conv2, and x2 T -> conv3).  Every layer's output is stored (the backward
// reads them all) and kept in LDS as the next layer's input, so no layer
// re-reads its input from HBM or waits out a launch boundary.  Per layer the
// same operations in the same order as k_pw_fwd3 / k_pw_fwd (conv1's fma
// chain; the k-permuted f32 MFMA chain, then + bias, then the activation), so
// every output is bitwise what the per-layer launches write.  Persistent:
// 2 workgroups per CU stride over the tiles, each keeping the shared weights'
// fragments in registers; a per-cloud weight (rows_per_w, the transform T) is
// re-fetched for the next tile right after its layer, in flight meanwhile.
// ---------------------------------------------------------------------------
// LDS row strides (floats, = 4 mod 64 banks): buffer 0 holds up to 128
// columns, buffer 1 up to 64 (52.2 KB in all: three workgroups per CU)
constexpr int PC_S0 = 132, PC_S1 = 68;
constexpr int PC_GRID = 768;
__host__ __device__ constexpr int pc_stride(int k) { return k ? PC_S1 : PC_S0; }

struct PwChainLayer {
  WView wv;
  const float* b;
  float* y;
  int act;
};
struct PwChainArgs {
  PwChainLayer l[PCADV_PW_CHAIN_MAX];
};
struct PwChainLds {
  alignas(16) float pts[PW_ROWS * 4];
  alignas(16) float buf0[PW_ROWS * PC_S0];
  alignas(16) float buf1[PW_ROWS * PC_S1];
  __device__ float* buf(int k) { return k ? buf1 : buf0; }
};

// B fragments of one K = 64 layer for this wave's 32-column tile (k_pw_fwd's
// loads; O = 64: columns 32 (wave & 1), O = 128: columns 32 wave).  KMAJ: the
// weight is a [K][O] matrix (coalesced 4-B loads across the lanes), else a
// 16-B aligned [O][K] one (the launcher checks the alignment)
template <int O, bool KMAJ>
__device__ __forceinline__ void chain_frags(const WView& wv, int r0, int wave, int lane,
                                            f32x4 (&bf)[8]) {
  const int r = lane & 31, h = lane >> 5;
  const int oc = O == 64 ? 32 * (wave & 1) : 32 * wave;
  const float* w = wv.base(r0);
  if constexpr (!KMAJ) {
#pragma unroll
    for (int g = 0; g < 8; ++g)
      bf[g] = *reinterpret_cast<const f32x4*>(w + (size_t)(oc + r) * 64 + 8 * g + 4 * h);
  } else {
    const float* c = w + (size_t)(4 * h) * O + oc + r;
#pragma unroll
    for (int g = 0; g < 8; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[g][j] = c[(size_t)(8 * g + j) * O];
  }
}

// one K = 64 layer of the tile on the f32 MFMA (k_pw_fwd's chain per output):
// in -> out, LDS [64][SI] -> [64][SO]
template <int O, int ACT, int SI, int SO>
__device__ __forceinline__ void chain_mfma(const float* in, float* out, const f32x4 (&bf)[8],
                                           float bias, int wave, int lane) {
  const int r = lane & 31;
  const int oc = O == 64 ? 32 * (wave & 1) : 32 * wave;
  const int rt0 = O == 64 ? (wave >> 1) : 0;
  constexpr int NRT = O == 64 ? 1 : 2;
#pragma unroll
  for (int t = 0; t < NRT; ++t) {
    const int rt = rt0 + t;
    f32x16 acc = {};
    acc = mfma_rows_x_wt<64>(in + 32 * rt * SI, SI, bf, acc, lane);
#pragma unroll
    for (int e = 0; e < 16; ++e)
      out[(32 * rt + acc_row(e, lane)) * SO + oc + r] = act_fwd(acc[e] + bias, ACT);
  }
}

// a layer's output tile (LDS) to HBM as 16-B row pieces
template <int O, int S>
__device__ __forceinline__ void chain_store(const float* src, float* __restrict__ y, int r0, int M,
                                            int tid) {
  constexpr int V = O / 4;
#pragma unroll
  for (int q = 0; q < PW_ROWS * V / PW_T; ++q) {
    const int e = tid + PW_T * q, row = e / V, c4 = e % V;
    const f32x4 v = *reinterpret_cast<const f32x4*>(src + row * S + 4 * c4);
    if (r0 + row < M) *reinterpret_cast<f32x4*>(y + (size_t)(r0 + row) * O + 4 * c4) = v;
  }
}

// RELU: bit i set = layer i applies the ReLU (else no activation), KMAJ: bit
// i set = layer i's weight is [K][O] (compile-time masks: no per-element
// branches in the epilogues, one load form per weight).  Layer i
// reads its input buffer (pts / buf[0] for i = 0, else buf[i & 1]) and writes
// buf[(i + 1) & 1].  The K = 64 layers' B fragments alternate between two
// register sets: layer i's set is loaded while layer i - 1 runs (the next
// tile's first MFMA layer's during this tile's last layer).
template <int K0, int O1, int O2, int O3, int O4, int RELU, int KMAJ>
__global__ void __launch_bounds__(PW_T, 2)
k_pw_chain(const float* __restrict__ x, int M, int ntiles, PwChainArgs a) {
  constexpr int Os[5] = {K0, O1, O2, O3, O4};
  constexpr int NL = O4 ? 4 : O3 ? 3 : O2 ? 2 : 1;
  static_assert(K0 == 3 || K0 == 64, "chain input: 3 or 64 channels");
  static_assert(K0 != 3 || O1 == 64, "a K = 3 first layer has 64 outputs");
  static_assert(NL % 2 == 0, "the fragment sets alternate by layer parity");
  static_assert(O2 == 0 || O1 == 64, "MFMA layers take K = 64");
  static_assert(O3 == 0 || O2 == 64, "MFMA layers take K = 64");
  static_assert(O4 == 0 || O3 == 64, "MFMA layers take K = 64");
  static_assert(O1 <= 64 && O3 <= 64, "buffer 1 (the even layers' outputs) holds 64 columns");
  constexpr int F = K0 == 3 ? 1 : 0;  // first MFMA layer
  extern __shared__ __attribute__((aligned(16))) char smem[];
  PwChainLds& L = *reinterpret_cast<PwChainLds*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31;
  const int t0 = blockIdx.x, stride = gridDim.x;

  // every kernel argument the loop reads, named once (kernarg loads up front)
  WView wv[NL];
  const float* bp[NL];
  float* yp[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    wv[i] = a.l[i].wv;
    bp[i] = a.l[i].b;
    yp[i] = a.l[i].y;
  }
  float bias[NL];
#pragma unroll
  for (int i = F; i < NL; ++i) {
    const int oc = Os[i + 1] == 64 ? 32 * (wave & 1) : 32 * wave;
    bias[i] = bp[i] ? bp[i][oc + r] : 0.f;
  }
  float c1[4] = {0.f, 0.f, 0.f, 0.f};  // K0 = 3: conv1's w[o][0..2], b[o] of column tid & 63
  if constexpr (K0 == 3) {
    const int o = tid & 63;
    const float* w = wv[0].base(t0 * PW_ROWS);
    c1[0] = wv[0].get(w, o, 0);
    c1[1] = wv[0].get(w, o, 1);
    c1[2] = wv[0].get(w, o, 2);
    c1[3] = bp[0] ? bp[0][o] : 0.f;
  }
  f32x4 fs[2][8];  // the two fragment sets
  constexpr bool kLastShares = ((NL - 1) & 1) == (F & 1);
  // layer i's fragments (i a constant once the layer loop is unrolled)
  auto frags = [&](int i, int rr, f32x4 (&bf)[8]) __attribute__((always_inline)) {
    const bool km = (KMAJ >> i) & 1;
    if (Os[i + 1] == 64 && km) chain_frags<64, true>(wv[i], rr, wave, lane, bf);
    if (Os[i + 1] == 64 && !km) chain_frags<64, false>(wv[i], rr, wave, lane, bf);
    if (Os[i + 1] == 128 && km) chain_frags<128, true>(wv[i], rr, wave, lane, bf);
    if (Os[i + 1] == 128 && !km) chain_frags<128, false>(wv[i], rr, wave, lane, bf);
  };
  frags(F, t0 * PW_ROWS, fs[F & 1]);

  // input tile: K0 = 3, thread < 192 holds one coordinate; K0 = 64, 16 floats
  // per thread as four 16-B pieces; rows past M read zeros
  f32x4 xin[K0 == 64 ? 4 : 1];
  auto load_in = [&](int tile) __attribute__((always_inline)) {
    const int r0 = tile * PW_ROWS;
    if constexpr (K0 == 3) {
      const int row = tid / 3;
      xin[0][0] = (tid < PW_ROWS * 3 && r0 + row < M) ? x[(size_t)r0 * 3 + tid] : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = tid + PW_T * j, row = e >> 4, c4 = e & 15;
        xin[j] = r0 + row < M ? *reinterpret_cast<const f32x4*>(x + (size_t)(r0 + row) * 64 + 4 * c4)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  load_in(t0);
  for (int tile = t0; tile < ntiles; tile += stride) {
    const int r0 = tile * PW_ROWS, nt = tile + stride;
    if constexpr (K0 == 3) {
      if (tid < PW_ROWS * 3) L.pts[(tid / 3) * 4 + tid % 3] = xin[0][0];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = tid + PW_T * j, row = e >> 4, c4 = e & 15;
        *reinterpret_cast<f32x4*>(&L.buf0[row * PC_S0 + 4 * c4]) = xin[j];
      }
    }
    __syncthreads();
    if (nt < ntiles) load_in(nt);  // in flight during this tile's layers
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      // the next MFMA layer's fragments (or the next tile's first) into the
      // other set: in flight while this layer runs
      if (i + 1 < NL) {
        if (i + 1 >= F) frags(i + 1, r0, fs[(i + 1) & 1]);
      } else if (nt < ntiles && !kLastShares) {
        frags(F, nt * PW_ROWS, fs[F & 1]);
      }
      float* out = L.buf((i + 1) & 1);
      const int so = pc_stride((i + 1) & 1);
      if (K0 == 3 && i == 0) {  // k_pw_fwd3's fma chain: thread = (column, 16 rows)
        const int o = tid & 63, rg = tid >> 6;
#pragma unroll 4
        for (int q = 0; q < 16; ++q) {
          const int row = 16 * rg + q;
          const float* p = &L.pts[row * 4];
          const float v = fmaf(c1[2], p[2], fmaf(c1[1], p[1], fmaf(c1[0], p[0], c1[3])));
          out[row * so + o] = act_fwd(v, (RELU & 1) ? ACT_RELU : ACT_NONE);
        }
      } else {
        const float* in = i == 0 ? L.buf0 : L.buf(i & 1);
        const int O = Os[i + 1];
        const bool relu = (RELU >> i) & 1;
        // buffer 1 (64 columns) is written by the even layers, read by the odd ones
        constexpr int A = ACT_RELU, N_ = ACT_NONE;
        const bool odd = i & 1;
        if (O == 64 && relu && !odd) chain_mfma<64, A, PC_S0, PC_S1>(in, out, fs[0], bias[i], wave, lane);
        if (O == 64 && !relu && !odd) chain_mfma<64, N_, PC_S0, PC_S1>(in, out, fs[0], bias[i], wave, lane);
        if (O == 64 && relu && odd) chain_mfma<64, A, PC_S1, PC_S0>(in, out, fs[1], bias[i], wave, lane);
        if (O == 64 && !relu && odd) chain_mfma<64, N_, PC_S1, PC_S0>(in, out, fs[1], bias[i], wave, lane);
        if (O == 128 && relu && odd) chain_mfma<128, A, PC_S1, PC_S0>(in, out, fs[1], bias[i], wave, lane);
        if (O == 128 && !relu && odd) chain_mfma<128, N_, PC_S1, PC_S0>(in, out, fs[1], bias[i], wave, lane);
      }
      // the last layer shares its set with the next tile's first MFMA layer:
      // that load goes out once this layer's MFMAs have read the set
      if (kLastShares && i + 1 == NL && nt < ntiles) frags(F, nt * PW_ROWS, fs[F & 1]);
      __syncthreads();
      if (Os[i + 1] == 64 && (i & 1)) chain_store<64, PC_S0>(out, yp[i], r0, M, tid);
      if (Os[i + 1] == 64 && !(i & 1)) chain_store<64, PC_S1>(out, yp[i], r0, M, tid);
      if (Os[i + 1] == 128) chain_store<128, PC_S0>(out, yp[i], r0, M, tid);
    }
    __syncthreads();  // the last copy-out and the input buffer's readers are done
  }
}

// ---------------------------------------------------------------------------
// backward, input gradient: dx[m][k] (+)= sum_o dz[m][o] w[o][k], dz = dy act'(y)
// ---------------------------------------------------------------------------
template <int R, int ACT>
__global__ void __launch_bounds__(PW_T)
k_pw_bwd_data(const float* __restrict__ dy, const float* __restrict__ yv, int M, WView wv,
              float* __restrict__ dx, int accumulate) {
  constexpr int SR = R + 4;
  __shared__ __attribute__((aligned(16))) float zs[PW_ROWS * SR];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * PW_ROWS, k0 = blockIdx.y * 128;
  const int K = wv.K;
  const float* w = wv.base(r0);
  for (int e = tid; e < PW_ROWS * R / 4; e += PW_T) {
    const int row = e / (R / 4), c4 = e % (R / 4);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r0 + row < M) {
      v = *reinterpret_cast<const f32x4*>(dy + (size_t)(r0 + row) * R + 4 * c4);
      if (ACT != ACT_NONE) {
        const f32x4 yy = *reinterpret_cast<const f32x4*>(yv + (size_t)(r0 + row) * R + 4 * c4);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= act_bwd(yy[j], ACT);
      }
    }
    *reinterpret_cast<f32x4*>(zs + row * SR + 4 * c4) = v;
  }
  __syncthreads();
  // wave -> (32-column tile, 32-row tiles): four column tiles over both row
  // tiles, or with K - k0 = 64 two column tiles x one row tile each (as in
  // k_pw_fwd), so every wave works; the same MFMA chain per output either way
  const bool narrow = K - k0 <= 64;
  const int kc = k0 + 32 * (narrow ? (wave & 1) : wave);
  if (kc >= K) return;  // K % 32 == 0
  const int rt0 = narrow ? (wave >> 1) : 0;
  const int r = lane & 31, h = lane >> 5;
  // B[o][k] = w[o][k]: lane (r, h) holds column kc + r at o = 8g + 4h + j
  f32x4 bf[R / 8];
  if (wv.kmajor && wv.aligned16()) {  // (o..o+3, k) contiguous: one 16-B load each
#pragma unroll
    for (int g = 0; g < R / 8; ++g)
      bf[g] = *reinterpret_cast<const f32x4*>(w + (size_t)(kc + r) * wv.O + 8 * g + 4 * h);
  } else {
#pragma unroll
    for (int g = 0; g < R / 8; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[g][j] = wv.get(w, 8 * g + 4 * h + j, kc + r);
  }
  const int col = kc + r;
  if (narrow) {
    f32x16 acc = {};
    acc = mfma_rows_x_wt<R>(zs + 32 * rt0 * SR, SR, bf, acc, lane);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ra = r0 + 32 * rt0 + acc_row(i, lane);
      if (ra < M) {
        float* p = dx + (size_t)ra * K + col;
        *p = accumulate ? *p + acc[i] : acc[i];
      }
    }
    return;
  }
  f32x16 acc0 = {}, acc1 = {};
  acc0 = mfma_rows_x_wt<R>(zs, SR, bf, acc0, lane);
  acc1 = mfma_rows_x_wt<R>(zs + 32 * SR, SR, bf, acc1, lane);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int ra = r0 + acc_row(i, lane), rb = ra + 32;
    if (ra < M) {
      float* p = dx + (size_t)ra * K + col;
      *p = accumulate ? *p + acc0[i] : acc0[i];
    }
    if (rb < M) {
      float* p = dx + (size_t)rb * K + col;
      *p = accumulate ? *p + acc1[i] : acc1[i];
    }
  }
}

// K = 3 (the points' gradient through a T-Net's conv1, STN3d models/pointnet.py:
// 28): thread = row, its three sums over o in ascending order (fma), W staged
// in LDS.  One weight matrix for all rows.
template <int R, int ACT>
__global__ void __launch_bounds__(PW_T)
k_pw_bwd_data3(const float* __restrict__ dy, const float* __restrict__ yv, int M, WView wv,
               float* __restrict__ dx, int accumulate) {
  __shared__ __attribute__((aligned(16))) float ws[R * 4];
  const int tid = threadIdx.x;
  for (int e = tid; e < R * 3; e += PW_T) ws[(e / 3) * 4 + e % 3] = wv.get(wv.w, e / 3, e % 3);
  __syncthreads();
  const int m = blockIdx.x * PW_T + tid;
  if (m >= M) return;
  const float* dyr = dy + (size_t)m * R;
  const float* yr = yv + (size_t)m * R;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll 4
  for (int o4 = 0; o4 < R / 4; ++o4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(dyr + 4 * o4);
    if (ACT != ACT_NONE) {
      const f32x4 yy = *reinterpret_cast<const f32x4*>(yr + 4 * o4);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= act_bwd(yy[j], ACT);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(ws + (4 * o4 + j) * 4);
      a0 = fmaf(v[j], w[0], a0);
      a1 = fmaf(v[j], w[1], a1);
      a2 = fmaf(v[j], w[2], a2);
    }
  }
  float* p = dx + (size_t)m * 3;
  p[0] = accumulate ? p[0] + a0 : a0;
  p[1] = accumulate ? p[1] + a1 : a1;
  p[2] = accumulate ? p[2] + a2 : a2;
}

// ---------------------------------------------------------------------------
// backward, weight gradient: per PWW_ROWS rows a slab of dW (O x K, layout
// [o][k] or [k][o]) and db (O)
// ---------------------------------------------------------------------------
template <int O, int K, int ACT>
__global__ void __launch_bounds__(PW_T)
k_pw_bwd_weight(const float* __restrict__ dy, const float* __restrict__ yv,
                const float* __restrict__ x, int M, int kmajor, float* __restrict__ slabs) {
  constexpr int SO = O + 32, SX = K + 32;  // row strides = 32 banks mod 64: conflict-free
  constexpr int NTILE = (O / 32) * (K / 32), NT = (NTILE + 3) / 4;
  __shared__ __attribute__((aligned(16))) float zs[PWW_SUB * SO];
  __shared__ __attribute__((aligned(16))) float xs[PWW_SUB * SX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int rbase = blockIdx.x * PWW_ROWS;
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
  float dbacc = 0.f;
  // the next 32 rows' operands are loaded into registers while the current
  // rows' MFMAs run (e = tid + PW_T * i covers each staging loop exactly)
  static_assert((PWW_SUB * O / 4) % PW_T == 0 && (PWW_SUB * K / 4) % PW_T == 0, "staging split");
  constexpr int NZ = PWW_SUB * O / 4 / PW_T, NX = PWW_SUB * K / 4 / PW_T;
  f32x4 pz[NZ], py[NZ], px[NX];
  auto load = [&](int r0) {
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      const int e = tid + PW_T * i, row = e / (O / 4), c4 = e % (O / 4);
      const bool in = r0 + row < M;
      const size_t off = (size_t)(in ? r0 + row : 0) * O + 4 * c4;
      pz[i] = in ? *reinterpret_cast<const f32x4*>(dy + off) : f32x4{0.f, 0.f, 0.f, 0.f};
      if (ACT != ACT_NONE) py[i] = *reinterpret_cast<const f32x4*>(yv + off);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int e = tid + PW_T * i, row = e / (K / 4), c4 = e % (K / 4);
      px[i] = r0 + row < M ? *reinterpret_cast<const f32x4*>(x + (size_t)(r0 + row) * K + 4 * c4)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  load(rbase);
  for (int sub = 0; sub < PWW_ROWS / PWW_SUB; ++sub) {
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      const int e = tid + PW_T * i, row = e / (O / 4), c4 = e % (O / 4);
      f32x4 v = pz[i];
      if (ACT != ACT_NONE) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= act_bwd(py[i][j], ACT);
      }
      *reinterpret_cast<f32x4*>(zs + row * SO + 4 * c4) = v;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int e = tid + PW_T * i, row = e / (K / 4), c4 = e % (K / 4);
      *reinterpret_cast<f32x4*>(xs + row * SX + 4 * c4) = px[i];
    }
    __syncthreads();
    if (sub + 1 < PWW_ROWS / PWW_SUB) load(rbase + (sub + 1) * PWW_SUB);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int tile = wave + 4 * t;
      if (tile < NTILE) {
        const int ot = tile / (K / 32), kt = tile % (K / 32);
        const float* ap = zs + h * SO + 32 * ot + r;
        const float* bp = xs + h * SX + 32 * kt + r;
#pragma unroll
        for (int s = 0; s < PWW_SUB / 2; ++s)
          acc[t] = mfma32(ap[2 * s * SO], bp[2 * s * SX], acc[t]);
      }
    }
    if (tid < O)
      for (int row = 0; row < PWW_SUB; ++row) dbacc += zs[row * SO + tid];
    __syncthreads();
  }
  float* slab = slabs + (size_t)blockIdx.x * (O * K + O);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tile = wave + 4 * t;
    if (tile < NTILE) {
      const int ot = tile / (K / 32), kt = tile % (K / 32);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int o = 32 * ot + acc_row(i, lane), k = 32 * kt + r;
        slab[kmajor ? k * O + o : o * K + k] = acc[t][i];
      }
    }
  }
  if (tid < O) slab[O * K + tid] = dbacc;
}

// K = 3 (conv1 weights over the points): thread = (o, quarter of the slab's
// rows), four accumulators (k = 0..2 and the bias); RB rows' operands loaded
// before their fmas; the quarters added in order through LDS
__global__ void __launch_bounds__(PW_T)
k_pw_bwd_weight3(const float* __restrict__ dy, const float* __restrict__ yv, int act,
                 const float* __restrict__ x, int M, int O, float* __restrict__ slabs) {
  __shared__ float part[4][64][4];
  const int tid = threadIdx.x, o = tid & 63, rq = tid >> 6;  // O <= 64
  const int rbase = blockIdx.x * PWW_ROWS + rq * (PWW_ROWS / 4);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (o < O) {
    constexpr int RB = 16;
    for (int i0 = 0; i0 < PWW_ROWS / 4; i0 += RB) {
      float z[RB], xv[RB][3];
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int m = rbase + i0 + u;
        const bool ok = m < M;
        const size_t mm = ok ? (size_t)m : 0;
        z[u] = ok ? dy[mm * O + o] : 0.f;
        if (act != ACT_NONE) z[u] *= ok ? act_bwd(yv[mm * O + o], act) : 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) xv[u][k] = ok ? x[mm * 3 + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < RB; ++u)
        if (rbase + i0 + u < M) {
#pragma unroll
          for (int k = 0; k < 3; ++k) acc[k] = fmaf(z[u], xv[u][k], acc[k]);
          acc[3] += z[u];
        }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) part[rq][o][k] = acc[k];
  __syncthreads();
  if (rq == 0 && o < O) {
    float* slab = slabs + (size_t)blockIdx.x * (O * 3 + O);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v = ((part[0][o][k] + part[1][o][k]) + part[2][o][k]) + part[3][o][k];
      if (k < 3) slab[o * 3 + k] = v;
      else slab[O * 3 + o] = v;
    }
  }
}

// out[g][j] = sum_{s < per} slabs[g*per + s][j] in a fixed order: 64 columns
// per block (one per lane), the 16 waves take contiguous slab ranges (8 loads
// in flight per lane), their partials added in wave order; j < W: dW, j = W.. : db
constexpr int PWR_W = 16;  // waves per reduce block
__global__ void __launch_bounds__(64 * PWR_W)
k_pw_reduce(const float* __restrict__ slabs, int per, int width, int wsize,
            float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float part[PWR_W][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane, g = blockIdx.y;
  const int s0 = wave * per / PWR_W, s1 = (wave + 1) * per / PWR_W;
  float acc = 0.f;
  if (j < width) {
    const float* s = slabs + (size_t)g * per * width + j;
    int i = s0;
    for (; i + 8 <= s1; i += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(i + u) * width];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; i < s1; ++i) acc += s[(size_t)i * width];
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && j < width) {
    float x = part[0][lane];
    for (int w = 1; w < PWR_W; ++w) x += part[w][lane];
    if (j < wsize) dw[(size_t)g * wsize + j] = x;
    else if (db) db[(size_t)g * (width - wsize) + j - wsize] = x;
  }
}

// Several weight gradients' slab sums in ONE launch (blockIdx.y = job), each
// job summed exactly as k_pw_reduce sums it (same slabs, order and waves), so
// the results are bitwise the per-gradient launches'.
constexpr int PWR_MAXJOBS = 8;
struct PwReduceJobs {
  const float* slabs[PWR_MAXJOBS];
  float* dw[PWR_MAXJOBS];
  float* db[PWR_MAXJOBS];
  int per[PWR_MAXJOBS], width[PWR_MAXJOBS], wsize[PWR_MAXJOBS];
};
__global__ void __launch_bounds__(64 * PWR_W) k_pw_reduce_batch(PwReduceJobs jb) {
  __shared__ float part[PWR_W][64];
  const int q = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = jb.per[q], width = jb.width[q];
  const int j = blockIdx.x * 64 + lane;
  if ((int)blockIdx.x * 64 >= width) return;  // block-uniform
  const int s0 = wave * per / PWR_W, s1 = (wave + 1) * per / PWR_W;
  float acc = 0.f;
  if (j < width) {
    const float* s = jb.slabs[q] + j;
    int i = s0;
    for (; i + 8 <= s1; i += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(i + u) * width];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; i < s1; ++i) acc += s[(size_t)i * width];
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && j < width) {
    float x = part[0][lane];
    for (int w = 1; w < PWR_W; ++w) x += part[w][lane];
    if (j < jb.wsize[q]) jb.dw[q][j] = x;
    else if (jb.db[q]) jb.db[q][j - jb.wsize[q]] = x;
  }
}

// ---------------------------------------------------------------------------
// conv + max over points, backward (sparse; optional ReLU before the max)
// ---------------------------------------------------------------------------
constexpr int CMB_PCH = 128;  // points per workgroup
constexpr int CMB_T = 512;
constexpr int CMB_MAXO = 1024;

struct CmbLds {
  int so[CMB_MAXO];
  float sg[CMB_MAXO];
  int okey[CMB_MAXO];
  float ogv[CMB_MAXO];
  int rcnt[CMB_PCH], fill[CMB_PCH], roff[CMB_PCH];
  int wsum[2];
};

__device__ __forceinline__ float cm_g(const float* dg, const float* gmax, size_t i) {
  const float g = dg[i];
  return gmax ? (gmax[i] > 0.f ? g : 0.f) : g;
}

// blocks [0, C * nchunk): dX rows of one (cloud, 128-point chunk); the rest:
// dW/db, one wave per output channel
__global__ void __launch_bounds__(CMB_T)
k_convmax_bwd(const float* __restrict__ dg, const int32_t* __restrict__ gidx,
              const float* __restrict__ gmax, const float* __restrict__ x, int C, int N, int K,
              const float* __restrict__ w, int O, float* __restrict__ dw, float* __restrict__ db,
              float* __restrict__ dx, int nchunk, int dx_relu) {
  __shared__ CmbLds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nxb = dx ? C * nchunk : 0;
  if ((int)blockIdx.x >= nxb) {
    // ---- dW[o,:] = sum_c g'[c,o] x[c, gidx[c,o], :], db[o] = sum_c g'[c,o]
    const int o = ((int)blockIdx.x - nxb) * 8 + wave;
    if (o >= O) return;
    // CB clouds' gradients, argmax rows and x rows in flight at once, summed
    // in cloud order (a cloud at a time was one dependent round trip each)
    constexpr int CB = 16;
    float a0 = 0.f, a1 = 0.f, ab = 0.f;
    for (int c0 = 0; c0 < C; c0 += CB) {
      float g[CB], v0[CB], v1[CB];
      int r[CB];
#pragma unroll
      for (int u = 0; u < CB; ++u) {
        const size_t i = (size_t)min(c0 + u, C - 1) * O + o;
        g[u] = c0 + u < C ? cm_g(dg, gmax, i) : 0.f;
        r[u] = gidx[i];
      }
#pragma unroll
      for (int u = 0; u < CB; ++u) {
        const float* row = x + ((size_t)min(c0 + u, C - 1) * N + r[u]) * K;
        v0[u] = lane < K ? row[lane] : 0.f;
        v1[u] = lane + 64 < K ? row[lane + 64] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < CB; ++u) {
        if (c0 + u < C) {
          a0 = fmaf(g[u], v0[u], a0);
          a1 = fmaf(g[u], v1[u], a1);
          ab += g[u];
        }
      }
    }
    if (lane < K) dw[(size_t)o * K + lane] = a0;
    if (lane + 64 < K) dw[(size_t)o * K + lane + 64] = a1;
    if (lane == 0 && db) db[o] = ab;
    return;
  }
  // ---- dX rows: hits (channels whose argmax is in the chunk) sorted by (row, o)
  const int c = blockIdx.x / nchunk, p0 = (blockIdx.x % nchunk) * CMB_PCH;
  if (tid < CMB_PCH) {
    L.rcnt[tid] = 0;
    L.fill[tid] = 0;
  }
  __syncthreads();
  constexpr int PER = CMB_MAXO / CMB_T;
  int hrow[PER];
  float hg[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int o = u * CMB_T + tid;
    const int a = o < O ? gidx[(size_t)c * O + o] : -1;
    // channels whose ReLU-before-max output is 0 carry no gradient: with the
    // ReLU every all-negative channel's argmax is point 0, hundreds of hits on
    // one row that one thread group would walk (they add exact zeros)
    const bool hit = a >= p0 && a < p0 + CMB_PCH && (!gmax || gmax[(size_t)c * O + o] > 0.f);
    hrow[u] = hit ? a - p0 : -1;
    hg[u] = hit ? cm_g(dg, gmax, (size_t)c * O + o) : 0.f;
    if (hit) atomicAdd(&L.rcnt[a - p0], 1);
  }
  __syncthreads();
  if (wave < 2) {
    const int cnt = L.rcnt[tid];
    int v = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(v, d);
      if (lane >= d) v += t;
    }
    if (lane == 63) L.wsum[wave] = v;
    L.roff[tid] = v - cnt;
  }
  __syncthreads();
  if (wave == 1) L.roff[tid] += L.wsum[0];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PER; ++u)
    if (hrow[u] >= 0) {
      const int p = L.roff[hrow[u]] + atomicAdd(&L.fill[hrow[u]], 1);
      L.okey[p] = u * CMB_T + tid;
      L.ogv[p] = hg[u];
    }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PER; ++u)
    if (hrow[u] >= 0) {
      const int o = u * CMB_T + tid, s0 = L.roff[hrow[u]], s1 = s0 + L.rcnt[hrow[u]];
      int rank = 0;
      for (int j = s0; j < s1; ++j) rank += L.okey[j] < o;
      L.so[s0 + rank] = o;
      L.sg[s0 + rank] = hg[u];
    }
  __syncthreads();
  // thread = (column k, group of 32 consecutive rows): the group's hits are
  // contiguous in (row, o) order, walked flat with HD W loads in flight; each
  // row's sum runs over its hits in o order (rows without hits -> 0)
  const int k = tid & 127, grp = tid >> 7;
  if (k >= K) return;
  constexpr int RG = CMB_PCH / 4, HD = 8;
  const int r0 = grp * RG, r1 = min(r0 + RG, N - p0);
  if (r1 <= r0) return;
  const int j1 = L.roff[r1 - 1] + L.rcnt[r1 - 1];
  float* drow = dx + ((size_t)c * N + p0) * K + k;
  // dx_relu: dx stored as the layer below's dz = dx * [x > 0] (x = relu(z) is
  // this conv's input), so its consumers read no activations for the mask
  const float* xrow = x + ((size_t)c * N + p0) * K + k;
  auto put = [&](int rr, float v) {
    if (dx_relu && v != 0.f && !(xrow[(size_t)rr * K] > 0.f)) v = 0.f;
    drow[(size_t)rr * K] = v;
  };
  int row = r0, rend = L.roff[r0] + L.rcnt[r0];
  float acc = 0.f;
  for (int j = L.roff[r0]; j < j1; j += HD) {
    float wv[HD];
#pragma unroll
    for (int u = 0; u < HD; ++u)
      wv[u] = j + u < j1 ? w[(size_t)L.so[j + u] * K + k] : 0.f;
#pragma unroll
    for (int u = 0; u < HD; ++u) {
      if (j + u < j1) {
        while (j + u >= rend) {  // row done: store it, move to the next
          put(row, acc);
          acc = 0.f;
          ++row;
          rend = L.roff[row] + L.rcnt[row];
        }
        acc = fmaf(L.sg[j + u], wv[u], acc);
      }
    }
  }
  for (; row < r1; ++row) {  // the last row with hits, then the rows after it
    put(row, acc);
    acc = 0.f;
  }
}

// ---------------------------------------------------------------------------
// feature_transform_regularizer: ||T T^T - I||_F per cloud and its gradient
// (2 * gscale / (B n_b)) (T T^T - I) T, stored or (accumulate) added into dT;
// norms (nullable) written in either mode; step_inc (nullable): block 0 also
// advances the step counter (the fused cls FT step's, ahead of its Adam)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_tnet_reg(const float* __restrict__ T, int B, int k, float* __restrict__ norms,
           const float* __restrict__ gscale, float* __restrict__ dT, int accumulate,
           int32_t* __restrict__ step_inc) {
  extern __shared__ float sm[];
  const int ks = k + 1;       // LDS row stride: row j's element l for 32 consecutive j
  float* t = sm;              //   hits 32 banks (stride k = 64 was one bank)
  float* a = sm + k * ks;     // k x k, same stride
  __shared__ double part[256];
  const int tid = threadIdx.x, b = blockIdx.x;
  const float* tb = T + (size_t)b * k * k;
  for (int e = tid; e < k * k; e += 256) t[(e / k) * ks + e % k] = tb[e];
  __syncthreads();
  double ss = 0.0;
  if (k == 64) {  // thread -> a 4 x 4 block of T T^T: 8 LDS reads per 16 fmas
    const int i0 = 4 * (tid >> 4), j0 = 4 * (tid & 15);
    float v[4][4] = {};
    for (int l = 0; l < 64; ++l) {
      float ti[4], tj[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ti[u] = t[(i0 + u) * ks + l];
        tj[u] = t[(j0 + u) * ks + l];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[u][q] = fmaf(ti[u], tj[q], v[u][q]);
    }
    // (the norm's f64 sum of squares runs in this blocked element order)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float d = v[u][q] - ((i0 + u) == (j0 + q) ? 1.f : 0.f);
        a[(i0 + u) * ks + j0 + q] = d;
        ss += (double)d * d;
      }
  } else {
    for (int e = tid; e < k * k; e += 256) {
      const int i = e / k, j = e % k;
      float v = 0.f;
      for (int l = 0; l < k; ++l) v = fmaf(t[i * ks + l], t[j * ks + l], v);
      v -= (i == j) ? 1.f : 0.f;
      a[i * ks + j] = v;
      ss += (double)v * v;
    }
  }
  part[tid] = ss;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) part[tid] += part[tid + s];
    __syncthreads();
  }
  const float n = (float)sqrt(part[0]);
  if (norms && tid == 0) norms[b] = n;
  if (step_inc && b == 0 && tid == 0) *step_inc += 1;
  if (!dT) return;
  const float scale = 2.f * (*gscale) / ((float)B * n);
  if (k == 64) {  // (T T^T - I) T in 4 x 4 blocks
    const int i0 = 4 * (tid >> 4), j0 = 4 * (tid & 15);
    float v[4][4] = {};
    for (int l = 0; l < 64; ++l) {
      float ai[4], tl[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ai[u] = a[(i0 + u) * ks + l];
        tl[u] = t[l * ks + j0 + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[u][q] = fmaf(ai[u], tl[q], v[u][q]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float* d = &dT[(size_t)b * k * k + (i0 + u) * k + j0 + q];
        *d = accumulate ? *d + scale * v[u][q] : scale * v[u][q];
      }
  } else {
    for (int e = tid; e < k * k; e += 256) {
      const int i = e / k, j = e % k;
      float v = 0.f;
      for (int l = 0; l < k; ++l) v = fmaf(a[i * ks + l], t[l * ks + j], v);
      dT[(size_t)b * k * k + e] = accumulate ? dT[(size_t)b * k * k + e] + scale * v : scale * v;
    }
  }
}

__global__ void k_mean(const float* __restrict__ v, int n, float* __restrict__ out) {
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += v[i];
    *out = (float)(s / n);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static WView make_view(const float* w, int O, int K, int kmajor, int rows_per_w) {
  return WView{w, O, K, kmajor, rows_per_w, (long long)O * K};
}

int launch_pw_fwd(const float* x, int M, int K, const float* w, const float* b, int O, int act,
                  int w_kmajor, int rows_per_w, float* y, hipStream_t s) {
  PC_REQUIRE(M > 0 && (K == 3 || K == 64 || K == 128) && O > 0 && O % 32 == 0,
             "pw_fwd: unsupported shape M=%d K=%d O=%d", M, K, O);
  PC_REQUIRE(act == ACT_NONE || act == ACT_RELU, "pw_fwd: act %d", act);
  PC_REQUIRE(rows_per_w == 0 || rows_per_w % PW_ROWS == 0,
             "pw_fwd: rows per weight matrix (%d) must be a multiple of %d", rows_per_w, PW_ROWS);
  const WView wv = make_view(w, O, K, w_kmajor, rows_per_w);
  const dim3 grid((M + PW_ROWS - 1) / PW_ROWS, (O + 127) / 128);
  if (K == 3) {
    if (act == ACT_RELU) hipLaunchKernelGGL(k_pw_fwd3<ACT_RELU>, grid, dim3(PW_T), 0, s, x, M, wv, b, y);
    else hipLaunchKernelGGL(k_pw_fwd3<ACT_NONE>, grid, dim3(PW_T), 0, s, x, M, wv, b, y);
  }
#define PW_CASE(KK, A)                                                                      \
  if (K == KK && act == A)                                                                 \
    hipLaunchKernelGGL((k_pw_fwd<KK, A>), grid, dim3(PW_T), 0, s, x, M, wv, b, y);
  PW_CASE(64, ACT_NONE) PW_CASE(64, ACT_RELU) PW_CASE(128, ACT_NONE) PW_CASE(128, ACT_RELU)
#undef PW_CASE
  PC_HIP_CHECK_LAUNCH("k_pw_fwd");
  return PCADV_OK;
}

// the chain shapes instantiated: the feature-transform extractor's two runs
template <int K0, int O1, int O2, int O3, int O4, int RELU, int KMAJ>
static int launch_chain(const float* x, int M, const PwChainArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_pw_chain<K0, O1, O2, O3, O4, RELU, KMAJ>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(PwChainLds)) != hipSuccess) {
      set_error("pw_chain: cannot reserve %zu bytes of LDS", sizeof(PwChainLds));
      return PCADV_EHIP;
    }
    attr = true;
  }
  const int ntiles = (M + PW_ROWS - 1) / PW_ROWS;
  hipLaunchKernelGGL((k_pw_chain<K0, O1, O2, O3, O4, RELU, KMAJ>), dim3(ntiles < PC_GRID ? ntiles : PC_GRID), dim3(PW_T),
                     sizeof(PwChainLds), s, x, M, ntiles, a);
  PC_HIP_CHECK_LAUNCH("k_pw_chain");
  return PCADV_OK;
}

int launch_pw_chain(const float* x, int M, int K, const pcadv_pw_layer* layers, int n,
                    hipStream_t s) {
  PC_REQUIRE(x && layers && M > 0 && n >= 1 && n <= PCADV_PW_CHAIN_MAX,
             "pw_chain: bad arguments (M=%d, %d layers)", M, n);
  PwChainArgs a{};
  int k = K;
  int O[PCADV_PW_CHAIN_MAX] = {0, 0, 0, 0};
  int relu = 0, kmaj = 0;
  for (int i = 0; i < n; ++i) {
    const pcadv_pw_layer& l = layers[i];
    PC_REQUIRE(l.w && l.y && l.O > 0, "pw_chain: layer %d: weight, output and O are required", i);
    PC_REQUIRE(l.act == ACT_NONE || l.act == ACT_RELU, "pw_chain: layer %d: act %d", i, l.act);
    PC_REQUIRE(l.rows_per_w == 0 || l.rows_per_w % PW_ROWS == 0,
               "pw_chain: layer %d: rows per weight matrix (%d) must be a multiple of %d", i,
               l.rows_per_w, PW_ROWS);
    a.l[i] = PwChainLayer{make_view(l.w, l.O, k, l.w_kmajor, l.rows_per_w), l.b, l.y, l.act};
    O[i] = l.O;
    relu |= (l.act == ACT_RELU) << i;
    kmaj |= (l.w_kmajor != 0) << i;
    // [O][K] weights are read as 16-B pieces (each matrix of a stack too)
    PC_REQUIRE(l.w_kmajor || ((reinterpret_cast<uintptr_t>(l.w) & 15) == 0 &&
                              (l.rows_per_w == 0 || (l.O * k) % 4 == 0)),
               "pw_chain: layer %d: an [O][K] weight must be 16-byte aligned", i);
    k = l.O;
  }
  if (K == 3 && n == 4 && O[0] == 64 && O[1] == 64 && O[2] == 64 && O[3] == 128 && relu == 15 &&
      kmaj == 0)
    return launch_chain<3, 64, 64, 64, 128, 15, 0>(x, M, a, s);
  if (K == 64 && n == 2 && O[0] == 64 && O[1] == 128 && relu == 2 && kmaj == 1)
    return launch_chain<64, 64, 128, 0, 0, 2, 1>(x, M, a, s);
  set_error("pw_chain: shape K=%d -> %d layers (%d, %d, %d, %d; ReLU mask %d, [K][O] mask %d) is "
            "not instantiated (3 -> 64, 64, 64, 128 all ReLU [O][K], and 64 -> 64 [K][O], 128 ReLU "
            "[O][K] are)", K, n, O[0], O[1], O[2], O[3], relu, kmaj);
  return PCADV_EINVAL;
}

int launch_pw_bwd_data(const float* dy, const float* y, int act, int M, int O, const float* w,
                       int K, int w_kmajor, int rows_per_w, float* dx, int accumulate,
                       hipStream_t s) {
  PC_REQUIRE(M > 0 && (O == 64 || O == 128) && K > 0 && (K % 32 == 0 || K == 3),
             "pw_bwd_data: unsupported shape M=%d O=%d K=%d", M, O, K);
  PC_REQUIRE(act == ACT_NONE || act == ACT_RELU, "pw_bwd_data: act %d", act);
  PC_REQUIRE(rows_per_w == 0 || rows_per_w % PW_ROWS == 0, "pw_bwd_data: rows per weight %d",
             rows_per_w);
  PC_REQUIRE(K != 3 || rows_per_w == 0, "pw_bwd_data: K=3 takes one weight matrix");
  PC_REQUIRE(act == ACT_NONE || y, "pw_bwd_data: the layer output is needed for act'");
  const WView wv = make_view(w, O, K, w_kmajor, rows_per_w);
  if (K == 3) {
    const dim3 g3((M + PW_T - 1) / PW_T);
#define PW_CASE3(R, A)                                                                     \
  if (O == R && act == A)                                                                  \
    hipLaunchKernelGGL((k_pw_bwd_data3<R, A>), g3, dim3(PW_T), 0, s, dy, y, M, wv, dx, accumulate);
    PW_CASE3(64, ACT_NONE) PW_CASE3(64, ACT_RELU) PW_CASE3(128, ACT_NONE) PW_CASE3(128, ACT_RELU)
#undef PW_CASE3
    PC_HIP_CHECK_LAUNCH("k_pw_bwd_data3");
    return PCADV_OK;
  }
  const dim3 grid((M + PW_ROWS - 1) / PW_ROWS, (K + 127) / 128);
#define PW_CASE(R, A)                                                                      \
  if (O == R && act == A)                                                                  \
    hipLaunchKernelGGL((k_pw_bwd_data<R, A>), grid, dim3(PW_T), 0, s, dy, y, M, wv, dx, accumulate);
  PW_CASE(64, ACT_NONE) PW_CASE(64, ACT_RELU) PW_CASE(128, ACT_NONE) PW_CASE(128, ACT_RELU)
#undef PW_CASE
  PC_HIP_CHECK_LAUNCH("k_pw_bwd_data");
  return PCADV_OK;
}

size_t pw_bwd_weight_workspace_bytes(int M, int O, int K) {
  const size_t nslab = (M + PWW_ROWS - 1) / PWW_ROWS;
  return nslab * (size_t)(O * K + O) * sizeof(float);
}

int launch_pw_bwd_weight(const float* dy, const float* y, int act, const float* x, int M, int O,
                         int K, int rows_per_group, int dw_kmajor, float* dw, float* db, void* ws,
                         size_t ws_bytes, hipStream_t s) {
  PC_REQUIRE(M > 0 && (O == 64 || O == 128) && (K == 3 || K == 64 || K == 128),
             "pw_bwd_weight: unsupported shape M=%d O=%d K=%d", M, O, K);
  PC_REQUIRE(act == ACT_NONE || act == ACT_RELU, "pw_bwd_weight: act %d", act);
  PC_REQUIRE(rows_per_group == 0 || (M % rows_per_group == 0 && rows_per_group % PWW_ROWS == 0),
             "pw_bwd_weight: rows per group %d must divide M=%d and be a multiple of %d",
             rows_per_group, M, PWW_ROWS);
  PC_REQUIRE(K != 3 || (!dw_kmajor && O <= 64), "pw_bwd_weight: K=3 needs O <= 64, [o][k]");
  PC_REQUIRE(ws && ws_bytes >= pw_bwd_weight_workspace_bytes(M, O, K),
             "pw_bwd_weight: workspace too small");
  PC_REQUIRE(dw || (!db && rows_per_group == 0 && !dw_kmajor),
             "pw_bwd_weight: the deferred form (dw = db = NULL) takes rows_per_group 0, [o][k]");
  float* slabs = static_cast<float*>(ws);
  const int nslab = (M + PWW_ROWS - 1) / PWW_ROWS;
  if (K == 3) {
    hipLaunchKernelGGL(k_pw_bwd_weight3, dim3(nslab), dim3(PW_T), 0, s, dy, y, act, x, M, O, slabs);
  } else {
#define PW_CASE(OO, KK, A)                                                                 \
  if (O == OO && K == KK && act == A)                                                      \
    hipLaunchKernelGGL((k_pw_bwd_weight<OO, KK, A>), dim3(nslab), dim3(PW_T), 0, s, dy, y, x, M, \
                       dw_kmajor, slabs);
    PW_CASE(64, 64, ACT_NONE) PW_CASE(64, 64, ACT_RELU) PW_CASE(64, 128, ACT_NONE)
    PW_CASE(64, 128, ACT_RELU) PW_CASE(128, 64, ACT_NONE) PW_CASE(128, 64, ACT_RELU)
    PW_CASE(128, 128, ACT_NONE) PW_CASE(128, 128, ACT_RELU)
#undef PW_CASE
  }
  PC_HIP_CHECK_LAUNCH("k_pw_bwd_weight");
  if (!dw) return PCADV_OK;  // slabs only: summed later by launch_pw_wgrad_finish
  const int width = O * K + O;
  const int groups = rows_per_group ? M / rows_per_group : 1;
  const int per = rows_per_group ? rows_per_group / PWW_ROWS : nslab;
  hipLaunchKernelGGL(k_pw_reduce, dim3((width + 63) / 64, groups), dim3(64 * PWR_W), 0, s, slabs,
                     per, width, O * K, dw, db);
  PC_HIP_CHECK_LAUNCH("k_pw_reduce");
  return PCADV_OK;
}

int launch_pw_wgrad_finish(const pcadv_pw_wgrad_job* jobs, int njobs, hipStream_t s) {
  PC_REQUIRE(jobs && njobs >= 1 && njobs <= PWR_MAXJOBS, "pw_wgrad_finish: %d jobs (1..%d)", njobs,
             PWR_MAXJOBS);
  PwReduceJobs jb{};
  int maxw = 0;
  for (int k = 0; k < njobs; ++k) {
    const pcadv_pw_wgrad_job& j = jobs[k];
    PC_REQUIRE(j.slabs && j.dw && j.M > 0 && (j.O == 64 || j.O == 128) &&
                   (j.K == 3 || j.K == 64 || j.K == 128),
               "pw_wgrad_finish: job %d: bad arguments (M=%d O=%d K=%d)", k, j.M, j.O, j.K);
    jb.slabs[k] = static_cast<const float*>(j.slabs);
    jb.dw[k] = j.dw;
    jb.db[k] = j.db;
    jb.per[k] = (j.M + PWW_ROWS - 1) / PWW_ROWS;
    jb.width[k] = j.O * j.K + j.O;
    jb.wsize[k] = j.O * j.K;
    if (jb.width[k] > maxw) maxw = jb.width[k];
  }
  hipLaunchKernelGGL(k_pw_reduce_batch, dim3((maxw + 63) / 64, njobs), dim3(64 * PWR_W), 0, s, jb);
  PC_HIP_CHECK_LAUNCH("k_pw_reduce_batch");
  return PCADV_OK;
}

int launch_convmax_bwd(const float* dg, const int32_t* gidx, const float* gmax, const float* x,
                       int C, int N, int K, const float* w, int O, float* dw, float* db,
                       float* dx, hipStream_t s, int dx_relu) {
  PC_REQUIRE(C > 0 && N > 0 && K > 0 && K <= 128 && O > 0 && O <= CMB_MAXO && dw,
             "convmax_bwd: unsupported shape C=%d N=%d K=%d O=%d", C, N, K, O);
  const int nchunk = (N + CMB_PCH - 1) / CMB_PCH;
  const int nxb = dx ? C * nchunk : 0;
  hipLaunchKernelGGL(k_convmax_bwd, dim3(nxb + (O + 7) / 8), dim3(CMB_T), 0, s, dg, gidx, gmax, x,
                     C, N, K, w, O, dw, db, dx, nchunk, dx_relu);
  PC_HIP_CHECK_LAUNCH("k_convmax_bwd");
  return PCADV_OK;
}

int launch_tnet_reg(const float* T, int B, int k, float* norms, float* reg,
                    const float* gscale, float* dT, hipStream_t s, int accumulate,
                    int32_t* step_inc) {
  PC_REQUIRE(B > 0 && k > 0 && k <= 64, "tnet_reg: unsupported B=%d k=%d", B, k);
  PC_REQUIRE(!dT || gscale, "tnet_reg: the gradient needs the upstream gradient");
  PC_REQUIRE(!reg || norms, "tnet_reg: the mean needs the per-cloud norms");
  const size_t lds = 2 * (size_t)k * (k + 1) * sizeof(float);
  hipLaunchKernelGGL(k_tnet_reg, dim3(B), dim3(256), lds, s, T, B, k, norms, dT ? gscale : nullptr,
                     dT, accumulate, step_inc);
  PC_HIP_CHECK_LAUNCH("k_tnet_reg");
  if (reg) {
    hipLaunchKernelGGL(k_mean, dim3(1), dim3(64), 0, s, norms, B, reg);
    PC_HIP_CHECK_LAUNCH("k_mean");
  }
  return PCADV_OK;
}

}  // namespace pcadv

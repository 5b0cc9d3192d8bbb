// PointNetfeat forward (models/pointnet.py:109-132, feature_transform=False) on
// gfx950 in two launches:
//
//   k_point_mlp   64-point tiles, two per workgroup: conv1 -> conv2 -> conv3
//                 (+ ReLU).  Only x3 (post-ReLU conv3, the operand of conv4,
//                 the exact re-evaluation and the backward) leaves the chip.
//     conv1 (3 -> 64)    VALU, in the fma order the backward's recompute uses
//     conv2 (64 -> 64)   v_mfma_f32_32x32x2_f32 (exact f32, k-ordered)
//     conv3 (64 -> 128)  six v_mfma_f32_32x32x16_bf16 products of three-way
//                        bf16 splits (f32-level accuracy)
//
//   k_conv4_max   one workgroup per (cloud, 256-channel block), weight-
//                 stationary: each of the 8 waves holds its 32 channels of W4 as
//                 bf16 hi + lo in registers and the cloud's points stream
//                 through LDS in 64-point steps (x3 f32 from L2/MALL, split to
//                 bf16 hi + lo once per workgroup).  conv4 runs as three
//                 v_mfma_f32_32x32x16_bf16 per product (x_hi w_hi + x_hi w_lo +
//                 x_lo w_hi, f32 accumulate; relative error <= ~1.2e-5 of
//                 sum|x w|) and the screening epilogue keeps each lane's top-2
//                 (value, point) over the whole cloud in registers.  The tail
//                 re-evaluates the winner and the runner-up as exact f32 dot
//                 products and ranks them by those, so gmax is f32 and the argmax follows
//                 the f32 values with the first index on ties (torch.max on
//                 CPU).  The 128 MB conv4 output never exists.
#include "common.h"

#include <type_traits>
#include <utility>

namespace pcadv {

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ============================================================================
// k_point_mlp: conv1..conv3
// ============================================================================
constexpr int PM_P = 64;    // points per tile
constexpr int PM_T = 256;   // 4 waves; 2 workgroups per CU (register-bound)
// TPW: tiles per workgroup (the next tile's points are prefetched): 2, or 1 when
// two would leave fewer than two workgroups per CU (fewer than 64 clouds at N = 1024)
constexpr int X2S = 72;     // bf16 row stride of the x2 planes (144 B: conflict-free b128 reads)

constexpr int X3S = 136;     // f32 row stride of the x3 store staging (the two half-waves' rows 32 banks apart)
// one tile per workgroup: the 64 x 128 conv3 tile staged over x1 / x2 for
// 512-B row stores
struct MlpLds1 {
  alignas(16) float pts[PM_P * 4];
  union {
    struct {
      alignas(16) float x1[PM_P * S64];
      alignas(16) __bf16 x2[3][PM_P * X2S];  // conv2 output split in bf16 hi / mid / lo
    };
    alignas(16) float x3[PM_P * X3S];  // the tile's conv3 output, staged for 16-B stores
  };
};
// two tiles per workgroup: each wave stages its own 64 x 32 slice of conv3's
// output (x3w[wave], no workgroup barrier), kept until its stores are issued
// during the next tile; 78.8 KB, two workgroups per CU
struct MlpLds2 {
  alignas(16) float pts[PM_P * 4];
  alignas(16) float x1[PM_P * S64];
  alignas(16) __bf16 x2[3][PM_P * X2S];
  alignas(16) float x3w[4][PM_P * 32];  // [wave][point][32 channels]
};
// (the folded-gather instantiation keeps the block staging: with the
// per-wave form it needs more than 256 VGPRs)
template <int TPW, bool FOLD>
constexpr bool kMlpWaveStage = TPW == 2 && !FOLD;

// bf16 mode's x3 store: eight staged f32 (16-B aligned) rounded to bf16 (nearest
// even, the rounding k_conv4_max applied to the f32 x3 before) as one 16-B
// nontemporal store
__device__ __forceinline__ void store_bf16x8(__bf16* dst, const float* src) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(src), b = *reinterpret_cast<const f32x4*>(src + 4);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (__bf16)a[j];
    o[j + 4] = (__bf16)b[j];
  }
  __builtin_nontemporal_store(__builtin_bit_cast(f32x4, o), reinterpret_cast<f32x4*>(dst));
}
template <int TPW, bool FOLD>
using MlpLds = std::conditional_t<kMlpWaveStage<TPW, FOLD>, MlpLds2, MlpLds1>;

// conv1 and conv2 run in exact f32 (VALU, then v_mfma_f32_32x32x2_f32 in the k
// order of mfma_rows_x_wt), bitwise what the backward recomputes.  conv3 runs
// on the bf16 matrix pipe as six products of the three-way splits of x2 and W3
// (h h, h m, m h, h l, m m, l h; the dropped m l, l m, l l terms are < 2^-23 of
// |x w|), f32 accumulate: f32-level accuracy at 6/16 of the f32 MFMA cycles.
// NP3: conv3's bf16 products per f32 product: 6 (f32-level, the default) or 1
// (bf16 mode: x2 and W3 rounded to bf16, f32 accumulate).
// FOLD: the input batches are gathered here (GatherFold, the trainer's graph)
// instead of read from pts_a / pts_b; a separate instantiation, so the plain
// kernel's code is unchanged.
template <int NP3, int TPW, bool FOLD>
__global__ void __launch_bounds__(PM_T) __attribute__((amdgpu_waves_per_eu(2)))
k_point_mlp(const float* __restrict__ pts_a, const float* __restrict__ pts_b, int split, int N,
            int T, int ntiles, const float* __restrict__ w1, const float* __restrict__ b1,
            const float* __restrict__ w2, const float* __restrict__ b2,
            const float* __restrict__ w3, const float* __restrict__ b3,
            float* __restrict__ x3g, int32_t* inc_counter, uint64_t* __restrict__ stamps,
            GatherFold gf) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  MlpLds<TPW, FOLD>& L = *reinterpret_cast<MlpLds<TPW, FOLD>*>(smem);
  constexpr bool WST = kMlpWaveStage<TPW, FOLD>;  // per-wave staging, stores during the next tile
#ifdef PCADV_STAMPS
  uint64_t* st = stamps + (size_t)blockIdx.x * 16;
#define STAMP(k) do { if (stamps && threadIdx.x == 0) st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP(k) do { } while (0)
#endif
  STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  if (inc_counter && tid == 0 && blockIdx.x == 0) *inc_counter += 1;

  // points of a tile: thread e < 192 holds one coordinate
  auto pts_load = [&](int tile) {
    const int c = tile / T, p0 = (tile % T) * PM_P;
    const float* pts = c < split ? pts_a + (size_t)c * N * 3 : pts_b + (size_t)(c - split) * N * 3;
    const int p = tid / 3;
    return (tid < PM_P * 3 && p0 + p < N) ? pts[(size_t)p0 * 3 + tid] : 0.f;
  };
  // the same, gathered here from the job's split at its device cursor with the
  // device jitter (as k_gather_clouds), the value also stored to the step's
  // input buffer (the backward's recompute reads it) and, in the cloud's first
  // tile, its label row; an out-of-range index leaves the buffer as it is
  auto pts_gather = [&](int tile) {
    const int c = tile / T, p0 = (tile % T) * PM_P;
    const pcadv_gather_job& j = gf.j[c < split ? 0 : 1];
    const int b = c < split ? c : c - split, p = p0 + tid / 3, d = tid % 3;
    if (!(tid < PM_P * 3 && p < N)) return 0.f;
    const int64_t src = j.order[(int64_t)*j.cursor * j.B + b];
    float* o = j.out + ((size_t)b * j.npts + p) * 3 + d;
    if (src < 0 || src >= j.n_src) return *o;
    const float x = j.src[((size_t)src * j.src_npts + p) * 3 + d];
    float v = x;
    if (j.sigma > 0.0) {
      const uint32_t st = j.step ? (uint32_t)*j.step : 0u;
      const int64_t tg = (int64_t)b * j.npts + p + j.rng_row0 * j.npts;
      v = jitter_coord(x, (float)j.sigma, (float)j.clip, jitter_normal(j.seed, st, tg, d));
    }
    *o = v;
    if (p0 == 0 && tid < j.lab_width && j.out_lab && j.src_lab)
      j.out_lab[(size_t)b * j.lab_width + tid] = j.src_lab[(size_t)src * j.lab_width + tid];
    return v;
  };
  auto pts_next = [&](int tile) {
    if constexpr (FOLD) return pts_gather(tile);
    else return pts_load(tile);
  };
  int tile = blockIdx.x * TPW;
  // loads in the order they are consumed (the memory counter waits in issue
  // order): the first tile's points and conv1's weights, then conv2's B
  // fragments; W3 after the first tile's conv1 (split three ways beside conv2's
  // MFMAs of the first tile)
  float pv = tile < ntiles ? pts_next(tile) : 0.f;
  // conv1: thread = (channel tid & 63, 16-point group tid >> 6)
  const int c1 = tid & 63, pg = tid >> 6;
  const float wa = w1[c1 * 3 + 0], wb = w1[c1 * 3 + 1], wc = w1[c1 * 3 + 2], bb1 = b1[c1];
  // (the scheduler otherwise issues conv2's fragments ahead of w1, so conv1
  // waits for them)
  __builtin_amdgcn_sched_barrier(0);
  // conv2: wave = (point tile wave >> 1, channel tile wave & 1), f32 B fragments
  f32x4 bf2[8];
  load_bfrag<64>(w2, 32 * (wave & 1), lane, bf2);
  const float bias2 = b2[32 * (wave & 1) + r];
  __builtin_amdgcn_sched_barrier(0);
  // conv3: wave = channel tile (32 channels), W3 rows split three ways:
  // lane (r, h) holds k = 16 kb + 8 h .. + 8 of channel 32 wave + r
  f32x4 w3raw[8];
  auto load_w3 = [&]() {
    const float* wrow = w3 + (size_t)(32 * wave + r) * 64 + 8 * h;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      w3raw[2 * kb] = *reinterpret_cast<const f32x4*>(wrow + 16 * kb);
      w3raw[2 * kb + 1] = *reinterpret_cast<const f32x4*>(wrow + 16 * kb + 4);
    }
  };
  const float bias3 = b3[32 * wave + r];
  bf16x8 w3h[4], w3m[4], w3l[4];
  auto split_w3 = [&]() {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 a, m, l;
        split3(j < 4 ? w3raw[2 * kb][j] : w3raw[2 * kb + 1][j - 4], a, m, l);
        w3h[kb][j] = a;
        w3m[kb][j] = m;
        w3l[kb][j] = l;
      }
  };
  STAMP(1);
  // pieces [u0, u1) of the wave's staged 64 x 32 slice of tile `stile` as 16-B
  // nontemporal stores: a tile's stores are issued during the next tile's
  // conv1 / conv2 (the last tile's at once), so the chip's x3 writes are not
  // one burst per tile
  auto store_x3 = [&](int stile, int u0, int u1) {
    const int sc = stile / T, sp0 = (stile % T) * PM_P;
    const float* xw = reinterpret_cast<const float*>(smem + offsetof(MlpLds2, x3w)) + wave * PM_P * 32;
    if constexpr (NP3 == 1) {  // bf16 mode: half the pieces, eight channels each
      __bf16* xb = reinterpret_cast<__bf16*>(x3g) + ((size_t)sc * N + sp0) * 128 + 32 * wave;
#pragma unroll
      for (int u = u0 / 2; u < u1 / 2; ++u) {
        const int e = lane + 64 * u, row = e >> 2, c8 = e & 3;
        if (sp0 + row < N) store_bf16x8(xb + (size_t)row * 128 + 8 * c8, &xw[row * 32 + 8 * c8]);
      }
      return;
    }
    float* xg = x3g + ((size_t)sc * N + sp0) * 128 + 32 * wave;
#pragma unroll
    for (int u = u0; u < u1; ++u) {
      const int e = lane + 64 * u, row = e >> 3, c4 = e & 7;
      if (sp0 + row < N)
        __builtin_nontemporal_store(*reinterpret_cast<const f32x4*>(&xw[row * 32 + 4 * c4]),
                                    reinterpret_cast<f32x4*>(xg + (size_t)row * 128 + 4 * c4));
    }
  };

  for (int it = 0; it < TPW && tile < ntiles; ++it, ++tile) {
    const int c = tile / T, p0 = (tile % T) * PM_P;
    if (tid < PM_P * 3) L.pts[(tid / 3) * 4 + tid % 3] = pv;
    __syncthreads();  // (also: every wave is past the previous tile's conv3 reads)
    STAMP(3 + 5 * it);
    if (it + 1 < TPW && tile + 1 < ntiles) pv = pts_next(tile + 1);  // in flight during this tile
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = pg * 16 + i;
      const f32x4 q = *reinterpret_cast<const f32x4*>(&L.pts[p * 4]);
      L.x1[p * S64 + c1] = conv1_point(wa, wb, wc, bb1, q.x, q.y, q.z);
    }
    // W3 issued only now: the prologue's in-order issue of its eight loads
    // would hold up conv1 (it lands during the barrier and conv2's MFMAs)
    if (it == 0) {
      __builtin_amdgcn_sched_barrier(0);
      load_w3();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (WST && it > 0) store_x3(tile - 1, 0, 4);
    __syncthreads();
    STAMP(4 + 5 * it);
    {  // conv2 + ReLU, written to LDS split three ways for conv3
      const int pt = wave >> 1, col = 32 * (wave & 1) + r;
      f32x16 acc = {};
      acc = mfma_rows_x_wt<64>(L.x1 + 32 * pt * S64, S64, bf2, acc, lane);
      // W3's split beside conv2's MFMAs of the first tile (conv1 does not wait
      // for W3 to land; the empty asm keeps the compiler from hoisting the
      // split, and with it the wait for W3, back into conv1)
      if (it == 0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) asm volatile("" : "+v"(w3raw[q]));
        split_w3();
      }
      if (WST && it > 0) store_x3(tile - 1, 4, 8);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float v = acc[i] + bias2;
        v = v > 0.f ? v : 0.f;
        const int row = 32 * pt + acc_row(i, lane);
        split3(v, L.x2[0][row * X2S + col], L.x2[1][row * X2S + col], L.x2[2][row * X2S + col]);
      }
    }
    __syncthreads();
    STAMP(5 + 5 * it);
    {  // conv3 (64 -> 128) + ReLU -> x3 (HBM): wave = channel tile, both point tiles
      f32x16 acc[2] = {{}, {}};
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const int off = (32 * pt + r) * X2S + 16 * kb + 8 * h;
          const bf16x8 xh = *reinterpret_cast<const bf16x8*>(&L.x2[0][off]);
          bf16x8 xm{}, xl{};
          if constexpr (NP3 == 6) {
            xm = *reinterpret_cast<const bf16x8*>(&L.x2[1][off]);
            xl = *reinterpret_cast<const bf16x8*>(&L.x2[2][off]);
          }
          if constexpr (NP3 == 6) {
            acc[pt] = mfma_bf16(xl, w3h[kb], acc[pt]);
            acc[pt] = mfma_bf16(xm, w3m[kb], acc[pt]);
            acc[pt] = mfma_bf16(xh, w3l[kb], acc[pt]);
            acc[pt] = mfma_bf16(xm, w3h[kb], acc[pt]);
            acc[pt] = mfma_bf16(xh, w3m[kb], acc[pt]);
          }
          acc[pt] = mfma_bf16(xh, w3h[kb], acc[pt]);
        }
      }
#ifdef PCADV_STAMPS
      asm volatile("s_nop 0" ::"v"(acc[0][0]), "v"(acc[1][15]));
#endif
      STAMP(6 + 5 * it);
      if constexpr (WST) {  // the wave's 64 x 32 slice through its own LDS rows, then
        // 128-B row pieces with 16-B nontemporal stores (as below)
        float* xw = L.x3w[wave];
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float v = acc[pt][i] + bias3;
            xw[(32 * pt + acc_row(i, lane)) * 32 + r] = v > 0.f ? v : 0.f;
          }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the last tile's stores now; the others' during the next tile (whose
        // conv3 rewrites these rows only after them)
        if (!(it + 1 < TPW && tile + 1 < ntiles)) store_x3(tile, 0, 8);
      } else {
      // stage the 64 x 128 tile through LDS (over x1 / x2: every wave is past
      // conv3's reads after the barrier), then write it as the contiguous 32 KB
      // it is in HBM with 16-B stores: a quarter of the store instructions.
      // Nontemporal: a cloud's tiles are written from all eight XCDs and read by
      // k_conv4_max on one, so lines left dirty in this XCD's L2 would only be
      // written back at the launch boundary (step -1.2 us in A/B)
      __syncthreads();
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = acc[pt][i] + bias3;
          L.x3[(32 * pt + acc_row(i, lane)) * X3S + 32 * wave + r] = v > 0.f ? v : 0.f;
        }
      __syncthreads();
      if constexpr (NP3 == 1) {  // bf16 mode: 16-B stores of eight channels
        __bf16* xb = reinterpret_cast<__bf16*>(x3g) + ((size_t)c * N + p0) * 128;
#pragma unroll
        for (int u = 0; u < PM_P * 16 / PM_T; ++u) {
          const int e = tid + PM_T * u, row = e >> 4, c8 = e & 15;
          if (p0 + row < N) store_bf16x8(xb + (size_t)row * 128 + 8 * c8, &L.x3[row * X3S + 8 * c8]);
        }
      } else {
      float* xg = x3g + ((size_t)c * N + p0) * 128;
#pragma unroll
      for (int u = 0; u < PM_P * 32 / PM_T; ++u) {
        const int e = tid + PM_T * u, row = e >> 5, c4 = e & 31;
        if (p0 + row < N)
          __builtin_nontemporal_store(*reinterpret_cast<const f32x4*>(&L.x3[row * X3S + 4 * c4]),
                                      reinterpret_cast<f32x4*>(xg + (size_t)row * 128 + 4 * c4));
      }
      }
      }
      STAMP(7 + 5 * it);
    }
  }
  STAMP(2);
#undef STAMP
}

// ============================================================================
// k_conv4_max: conv4 (128 -> 1024) + max over points
// ============================================================================
#ifndef PCADV_C4_CERT
// diagnostic builds only (make ab ABDEFS=-DPCADV_C4_CERT=1): every lane also
// tracks the largest screened key it DROPS (the channel's third candidate),
// and after the exact re-evaluation a channel is counted when that third value
// plus a rigorous screening-error bound reaches the winner's exact value -
// what certifying the argmax would have to re-check (tools/cert_diag.py)
#define PCADV_C4_CERT 0
#endif
#if PCADV_C4_CERT
// [0] channels counted, [1] channels seen, [2] channels whose third screened
// value lies within 2^-16 x the bound (an empirical band), [3] launches
__device__ unsigned int g_c4_cert[4];
#endif
#ifndef PCADV_C4_DIAG
#define PCADV_C4_DIAG 0  // diagnostic builds only: 1 = no screening, 2 = no staging
#endif
constexpr int C4_O = 1024;  // conv4 output channels
constexpr int C4_CB = 256;  // channels per workgroup (8 waves x 32)
constexpr int C4_T = 512;
constexpr int C4_P = 64;    // points per step
constexpr int C4_SB = 136;  // bf16 row stride of the x3 hi / lo tiles (272 B: conflict-free b128 reads)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int C4_WS = 132;  // f32 row stride of the prologue's W4 staging (conflict-free b128 reads)
union C4Lds {
  alignas(16) __bf16 x[2][2][2 * C4_P * C4_SB];  // x3 tiles [buffer][hi, lo], up to 128 rows
  alignas(16) float w[8][32 * C4_WS];        // prologue only: each wave's 32 rows of W4
};


// Screening keys: the f32 value mapped to an order-preserving int32 whose low
// 6 bits are replaced by 63 - (the point's row inside its 64-point step, less
// the lane-half offset 4 h), so v_max_i32 / v_med3_i32 keep the top-2 (value,
// row) of a lane with the lower row first on equal truncated values.  The 6
// dropped bits (2^-17 relative) only order the candidates, which the exact
// re-evaluation then ranks by their f32 values; NaN maps above +inf as
// torch.max ranks it.
__device__ __forceinline__ int screen_key(float v, int lowc) {
  const int b = __float_as_int(v);
  const int ord = b ^ ((b >> 31) & 0x7fffffff);  // int order == float order
  return (ord & ~63) | lowc;
}
// The same key in three instructions (hipcc spends four): t = sign smear;
// x = b ^ (t & 0x7fffffc0) (order-preserving except in the low bits, which
// are replaced); key = (x & ~63) | LOWC.  v_bitop3 table index = 4 S0 + 2 S1 + S2.
// Only for accumulators whose MFMAs retired several instructions earlier
// (inline asm is outside the compiler's MFMA hazard tracking).
template <int LOWC>
__device__ __forceinline__ int screen_key_asm(float v, int m_ord, int m_hi) {
  int t;
#if PCADV_C4_DIAG & 4  // diagnostic builds only: one instruction, order wrong for negative values
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=&v"(t) : "v"(v), "s"(m_hi), "n"(LOWC));
  (void)m_ord;
  return t;
#endif
  asm("v_ashrrev_i32 %0, 31, %1\n\t"
      "v_bitop3_b32 %0, %1, %0, %2 bitop3:0x78\n\t"
      "v_bitop3_b32 %0, %0, %3, %4 bitop3:0xea"
      : "=&v"(t)
      : "v"(v), "s"(m_ord), "s"(m_hi), "n"(LOWC));
  return t;
}
// push acc element I (row acc_row(I, 0) of the unit, plus 4 h) into a lane's
// top-2 (TOP2) or top-1 (bf16 mode, whose result is the screened winner itself)
template <int I, bool TOP2>
__device__ __forceinline__ void screen_one(const f32x16& acc, int m_ord, int m_hi, int& k1,
                                           int& k2, int& k3) {
  const int key = screen_key_asm<31 - ((I & 3) + 8 * (I >> 2))>(acc[I], m_ord, m_hi);
  if constexpr (PCADV_C4_CERT && TOP2) k3 = max(min(key, k2), k3);  // the key k2 / key drops
  if constexpr (TOP2) k2 = max(min(key, k1), k2);  // median(key, k1, k2) for k2 <= k1: v_med3_i32
  k1 = max(k1, key);
}
template <int I0, bool TOP2, int... J>
__device__ __forceinline__ void screen_seq(const f32x16& acc, int m_ord, int m_hi, int& k1,
                                           int& k2, int& k3, std::integer_sequence<int, J...>) {
  (screen_one<I0 + J, TOP2>(acc, m_ord, m_hi, k1, k2, k3), ...);
}
__device__ __forceinline__ int key_row(int k) { return 31 - (k & 63); }
__device__ __forceinline__ float key_value(int k) {
  const int ord = k & ~63;
  return __int_as_float(ord ^ ((ord >> 31) & 0x7fffffff));
}
constexpr int KEY_NONE = (int)0x80000000;  // below every real key

// Sum over the 32 lanes of each half-wave, the total in every lane of the half
// (DPP quad / half-row / row mirrors, then one swizzle across the two rows);
// every lane adds the same operands, so all get bitwise the same total.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
// Sum over each octet of lanes (8 k .. 8 k + 7), the total in all eight
__device__ __forceinline__ float octet_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
  v += dpp<0x141>(v);  // row_half_mirror: lane i <- 7 - i within 8 (the other quad)
  return v;
}
__device__ __forceinline__ float half_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
  v += dpp<0x141>(v);  // row_half_mirror: lane i <- 7 - i within 8 (the other quad)
  v += dpp<0x140>(v);  // row_mirror: lane i <- 15 - i within 16 (the other 8)
  v += __shfl_xor(v, 16);
  return v;
}

// (va, ia) ranks before (vb, ib): larger value, NaN above all, lower index on ties
__device__ __forceinline__ bool ranks_before(float va, int ia, float vb, int ib) {
  const bool na = va != va, nb = vb != vb;
  if (na || nb) return na && (!nb || ia < ib);
  return va > vb || (va == vb && ia < ib);
}

// Merge one step's top-2 keys (n1 >= n2, both tagged with step u) into the
// running top-2 (r1 >= r2, tags t1, t2) of earlier steps.  Keys of different
// steps compare by their truncated value only (the low bits are rows within a
// step): on equal values the earlier step, i.e. the lower point index, stays.
template <bool TOP2 = true>
__device__ __forceinline__ void pair_merge(int n1, int u1, int n2, int u2, int& r1, int& t1,
                                           int& r2, int& t2) {
  if constexpr (!TOP2) {  // top-1: the earlier step keeps equal truncated values
    const bool a = (n1 & ~63) > (r1 & ~63);
    r1 = a ? n1 : r1;
    t1 = a ? u1 : t1;
    return;
  }
  const int m1 = n1 & ~63, m2 = n2 & ~63, q1 = r1 & ~63, q2 = r2 & ~63;
  const bool a = m1 > q1;
  const int sa = q1 >= m2 ? r1 : n2;
  const int ta = q1 >= m2 ? t1 : u2;
  const int sb = q2 >= m1 ? r2 : n1;
  const int tb = q2 >= m1 ? t2 : u1;
  r2 = a ? sa : sb;
  t2 = a ? ta : tb;
  r1 = a ? n1 : r1;
  t1 = a ? u1 : t1;
}

// NP4: conv4's bf16 products per f32 product: 3 (f32-level screening + the exact
// f32 re-evaluation of the top two, the default) or 1 (bf16 mode: x3 and W4
// rounded to bf16, f32 accumulate; the screened winner is the result, no
// re-evaluation: gmax carries the 2^-17 key truncation).
// G2: fewer than 64 clouds leave CUs idle with 256-channel workgroups, so a
// workgroup takes 128 channels (8 per cloud) and its two wave groups (waves
// 0-3, 4-7: the same 32-channel blocks) screen alternate 32-point units of the
// same staged tiles; group 1 hands its top-2 to group 0 through LDS before the
// exact re-evaluation.  Still two waves per SIMD (a lone wave gets half the
// throughput: 4-wave workgroups measured slower).
// XB (bf16 mode only): x3 arrives as bf16 (k_point_mlp<1>'s store, the same
// rounding this kernel applies to an f32 x3), so the staging is a copy: half
// the bytes and none of the conversion the channel-block workgroups of a cloud
// would each redo.  With G2, XB workgroups run FOUR wave groups (16 waves,
// 128-point steps, units 4 s + grp): the bf16 staging fits twice the rows in
// the same LDS, W4 needs no lo fragments, and half as many step barriers are
// shared by twice the waves.
#ifndef PCADV_C4_G4
#define PCADV_C4_G4 1  // A/B builds: 0 = XB workgroups keep two wave groups
#endif
template <int NP4, bool G2, bool XB>
constexpr int c4_groups() { return G2 ? (XB && PCADV_C4_G4 ? 4 : 2) : 1; }
template <int NP4, bool G2, bool XB>
constexpr int c4_threads() { return c4_groups<NP4, G2, XB>() == 4 ? 2 * C4_T : C4_T; }

// P128 (the 256-channel form, N % 128 == 0): 128-point steps, four units per
// wave and step, two staged rows per thread: half the step barriers.
#ifndef PCADV_C4_P128
#define PCADV_C4_P128 1  // A/B builds: 0 = 64-point steps throughout
#endif
template <int NP4, bool G2, bool XB = false, bool P128 = false>
__global__ void __launch_bounds__((c4_threads<NP4, G2, XB>()))
k_conv4_max(const float* __restrict__ x3g, int C, int N, const float* __restrict__ w4,
            const float* __restrict__ b4, float* __restrict__ gmax, int32_t* __restrict__ gidx,
            uint64_t* __restrict__ stamps, int relu) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  C4Lds& L = *reinterpret_cast<C4Lds*>(smem);
  // XCD-aware order: consecutive workgroup ids run on different XCDs, so the
  // ids are remapped to keep the 4 channel blocks of a cloud on one XCD (they
  // stream the same x3 through that XCD's L2)
  int bid = blockIdx.x;
  const int nwg = gridDim.x;
  if ((nwg & 7) == 0) bid = (bid & 7) * (nwg >> 3) + (bid >> 3);
  const int c = G2 ? bid >> 3 : bid >> 2, cb = G2 ? bid & 7 : bid & 3;
#ifdef PCADV_STAMPS
  uint64_t* st = stamps + (size_t)blockIdx.x * 16;
#define STAMP(k) do { if (stamps && threadIdx.x == 0) st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP(k) do { } while (0)
#endif
  STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  constexpr int NGRP = c4_groups<NP4, G2, XB>();
  static_assert(!(P128 && G2), "P128 is the 256-channel form's");
  constexpr int UPS = G2 ? 1 : (P128 ? 4 : 2);  // units per wave and step
  constexpr int P = G2 ? 32 * NGRP : 32 * UPS;  // points per step
  constexpr int RPT = P * 8 / c4_threads<NP4, G2, XB>();  // staged rows per thread (1, or 2 at P128)
  const int wblk = G2 ? wave & 3 : wave;  // 32-channel block of this wave
  const int grp = G2 ? wave >> 2 : 0;     // G2: wave group = unit of each step
  constexpr int CB = G2 ? C4_CB / 2 : C4_CB;
  const int o = cb * CB + 32 * wblk + r;  // this lane's output channel
  static_assert(!XB || NP4 == 1, "a bf16 x3 is bf16 mode's");
  const float* xc = x3g + (size_t)c * N * 128;
  const __bf16* xcb = reinterpret_cast<const __bf16*>(x3g) + (size_t)c * N * 128;
  const int S = (N + P - 1) / P;

  // staging map: thread = (row tid >> 3, 16 consecutive k at 16 (tid & 7));
  // rows past the cloud re-read its last row (screening masks them)
  const int srow = tid >> 3, sk = 16 * (tid & 7);
  f32x4 stg[4 * RPT];
  bf16x8 stgb[2 * RPT];  // XB
  auto stage_load = [&](int s) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int p = min(s * P + srow + 64 * q, N - 1);
      if constexpr (XB) {
        const bf16x8* src = reinterpret_cast<const bf16x8*>(xcb + (size_t)p * 128 + sk);
        stgb[2 * q] = src[0];
        stgb[2 * q + 1] = src[1];
      } else {
        const f32x4* src = reinterpret_cast<const f32x4*>(xc + (size_t)p * 128 + sk);
#pragma unroll
        for (int j = 0; j < 4; ++j) stg[4 * q + j] = src[j];
      }
    }
  };
  float cert_ss = 0.f, cert_xn2 = 0.f;  // PCADV_C4_CERT >= 2: max_p ||x_p||^2 of the cloud
  auto cert_row_done = [&]() {
    if constexpr (PCADV_C4_CERT >= 2) {
      cert_xn2 = fmaxf(cert_xn2, octet_sum(cert_ss));
      cert_ss = 0.f;
    }
  };
  auto stage_write = [&](int buf) {  // split the staged f32 rows into bf16 hi / lo
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      bf16x8* dh = reinterpret_cast<bf16x8*>(&L.x[buf][0][(srow + 64 * q) * C4_SB + sk]);
      bf16x8* dl = reinterpret_cast<bf16x8*>(&L.x[buf][1][(srow + 64 * q) * C4_SB + sk]);
      if constexpr (XB) {
        dh[0] = stgb[2 * q];
        dh[1] = stgb[2 * q + 1];
        continue;
      }
      bf16x8 hi[2], lo[2];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float v = stg[4 * q + (j >> 2)][j & 3];
        if constexpr (PCADV_C4_CERT >= 2) cert_ss = fmaf(v, v, cert_ss);
        const __bf16 hb = (__bf16)v;
        hi[j >> 3][j & 7] = hb;
        lo[j >> 3][j & 7] = (__bf16)(v - (float)hb);
      }
      dh[0] = hi[0];
      dh[1] = hi[1];
      if constexpr (NP4 == 3) {
        dl[0] = lo[0];
        dl[1] = lo[1];
      }
    }
  };
  stage_load(0);
  // W4 rows of this wave's 32 channels: coalesced 1 KB loads into the wave's
  // own LDS rows (no workgroup barrier: only this wave reads them back), then
  // each lane takes k = 16 kb + 8 h .. + 8 of its channel, split to bf16 hi / lo
  bf16x8 bh[8], bl[8];
  {
    // four groups: group 0's waves stage the four channel blocks, every wave
    // reads its block's rows after a workgroup barrier
    const float* wsrc = w4 + (size_t)(cb * CB + 32 * wblk) * 128;
    float* wl = L.w[NGRP == 4 ? wblk : wave];
    if (NGRP != 4 || grp == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int e = 4 * (lane + 64 * i);  // float index in the 32 x 128 block
        *reinterpret_cast<f32x4*>(wl + (e >> 7) * C4_WS + (e & 127)) =
            *reinterpret_cast<const f32x4*>(wsrc + e);
      }
    }
    if constexpr (NGRP == 4) {
      __syncthreads();
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const float* wrow = wl + r * C4_WS + 8 * h;
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const f32x4 u0 = *reinterpret_cast<const f32x4*>(wrow + 16 * kb);
      const f32x4 u1 = *reinterpret_cast<const f32x4*>(wrow + 16 * kb + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? u0[j] : u1[j - 4];
        const __bf16 hb = (__bf16)v;
        bh[kb][j] = hb;
        bl[kb][j] = (__bf16)(v - (float)hb);
      }
    }
  }
  __syncthreads();  // every wave holds its fragments before tile 0 overwrites the staging rows
  stage_write(0);
  cert_row_done();
  stage_load(1);
  __syncthreads();
  STAMP(1);

  // Running top-2 keys of this lane (r1 >= r2) and the 32-point units they came
  // from.  Low key bits of acc element i: 31 - acc_row(i, 0), a compile-time
  // constant; the lane's rows are acc_row(i, 0) + 4 h and are decoded with the
  // lane's own h (keys are only compared within a lane).
  int r1 = KEY_NONE, r2 = KEY_NONE;
  int t1 = -1, t2 = -1;
  int r3 = KEY_NONE;  // PCADV_C4_CERT: the largest truncated key this lane dropped
  auto screen_unit = [&](const f32x16& acc, int u, auto MASKED, int kb_lo, int kb_hi, int& k1,
                         int& k2, int& k3) {
#pragma unroll
    for (int i = 2 * kb_lo; i < 2 * kb_hi; ++i) {
      if constexpr (decltype(MASKED)::value)
        if (u * 32 + acc_row(i, lane) >= N) continue;
      const int key = screen_key(acc[i], 31 - acc_row(i, 0));
      if constexpr (PCADV_C4_CERT && NP4 == 3) k3 = max(min(key, k2), k3);
      if constexpr (NP4 == 3) k2 = max(min(key, k1), k2);  // median(key, k1, k2): v_med3_i32
      k1 = max(k1, key);
    }
  };
  // unmasked screening of acc elements [I, I + CNT) with the asm keys
  const int m_ord = 0x7fffffc0, m_hi = ~63;
  auto screen_fast = [&](const f32x16& acc, auto I, auto CNT, int& k1, int& k2, int& k3) {
    screen_seq<decltype(I)::value, NP4 == 3>(acc, m_ord, m_hi, k1, k2, k3,
                                             std::make_integer_sequence<int, decltype(CNT)::value>{});
  };
  // PCADV_C4_CERT: a unit's top-2 (n1 >= n2) and dropped max n3 merged into the
  // running r1, r2, r3: the third largest of {n1, n2, r1, r2} is dropped too
  auto cert_merge = [&](int n1, int n2, int n3) {
    if constexpr (PCADV_C4_CERT && NP4 == 3) {
      const int m1 = n1 & ~63, m2 = n2 & ~63, q1 = r1 & ~63, q2 = r2 & ~63;
      r3 = max(r3, max(n3 & ~63, max(min(m1, q2), min(m2, q1))));
    }
  };

  // Software pipeline over 32-point units (step s, half pt): the 24 MFMAs of a
  // unit are issued in the same scheduling regions as the screening of the
  // previous unit (the other accumulator) and a share of the staging work, so
  // one wave's matrix and vector work overlap.
  f32x16 accA = {}, accB = {};  // units of half 0 / half 1 of a step
  auto unit = [&](int s, int pt, f32x16& cur, const f32x16& prev, auto SCREEN, auto MASKED) {
    const int buf = s & 1;
    const __bf16* xh = &L.x[buf][0][(32 * pt + r) * C4_SB + 8 * h];
    const __bf16* xl = &L.x[buf][1][(32 * pt + r) * C4_SB + 8 * h];
    const int uprev = G2 ? NGRP * s + pt - NGRP : UPS * s + pt - 1;
    // this unit's share of the staging: row q = pt of the thread's rows (G2: its one row)
    const bool stg_turn = G2 || pt < RPT;
    const int q = G2 ? 0 : (pt < RPT ? pt : 0);
    int k1 = KEY_NONE, k2 = KEY_NONE, k3 = KEY_NONE;
    bf16x8 fa[3][2];  // A fragments, a 3-deep register ring: [k-block % 3][hi, lo]
    auto frag = [&](int kb) {
      fa[kb % 3][0] = *reinterpret_cast<const bf16x8*>(xh + 16 * kb);
      if constexpr (NP4 == 3) fa[kb % 3][1] = *reinterpret_cast<const bf16x8*>(xl + 16 * kb);
    };
    frag(0);
    frag(1);
    cur = f32x16{};
    bf16x8 shi[2], slo[2];
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      __builtin_amdgcn_sched_barrier(0);
      if (kb + 2 < 8) frag(kb + 2);  // two k-blocks (six MFMAs) ahead of its use
      const bf16x8 ah = fa[kb % 3][0];
      const bf16x8 al = NP4 == 3 ? fa[kb % 3][1] : bf16x8{};
      if constexpr (NP4 == 3) {
        cur = mfma_bf16(al, bh[kb], cur);
        cur = mfma_bf16(ah, bl[kb], cur);
      }
      cur = mfma_bf16(ah, bh[kb], cur);
      if constexpr (decltype(SCREEN)::value && decltype(MASKED)::value) {
        screen_unit(prev, uprev, MASKED, kb, kb + 1, k1, k2, k3);
        asm volatile("" ::"v"(k1), "v"(k2));
      } else if constexpr (decltype(SCREEN)::value && !(PCADV_C4_DIAG & 1)) {
        // 16 values over k-blocks 1..7 (2,2,2,2,2,3,3); none in k-block 0, so the
        // previous unit's MFMAs have retired before the asm reads them
        // (tools/check_asm_hazards.py checks the distance in the ISA)
        using IC = std::integral_constant<int, 0>;
        if constexpr (NP4 == 3 || !P128) {
          if (kb == 1) screen_fast(prev, IC{}, std::integral_constant<int, 2>{}, k1, k2, k3);
          if (kb == 2) screen_fast(prev, std::integral_constant<int, 2>{}, std::integral_constant<int, 2>{}, k1, k2, k3);
          if (kb == 3) screen_fast(prev, std::integral_constant<int, 4>{}, std::integral_constant<int, 2>{}, k1, k2, k3);
          if (kb == 4) screen_fast(prev, std::integral_constant<int, 6>{}, std::integral_constant<int, 2>{}, k1, k2, k3);
          if (kb == 5) screen_fast(prev, std::integral_constant<int, 8>{}, std::integral_constant<int, 2>{}, k1, k2, k3);
          if (kb == 6) screen_fast(prev, std::integral_constant<int, 10>{}, std::integral_constant<int, 3>{}, k1, k2, k3);
          if (kb == 7) screen_fast(prev, std::integral_constant<int, 13>{}, std::integral_constant<int, 3>{}, k1, k2, k3);
        } else {
          // bf16 mode's P128 form: one MFMA per k-block and back-to-back units,
          // so k-blocks 0 and 1 stand between the previous unit's last MFMA
          // and the first read
          if (kb == 2) screen_fast(prev, IC{}, std::integral_constant<int, 3>{}, k1, k2, k3);
          if (kb == 3) screen_fast(prev, std::integral_constant<int, 3>{}, std::integral_constant<int, 3>{}, k1, k2, k3);
          if (kb == 4) screen_fast(prev, std::integral_constant<int, 6>{}, std::integral_constant<int, 3>{}, k1, k2, k3);
          if (kb == 5) screen_fast(prev, std::integral_constant<int, 9>{}, std::integral_constant<int, 3>{}, k1, k2, k3);
          if (kb == 6) screen_fast(prev, std::integral_constant<int, 12>{}, std::integral_constant<int, 2>{}, k1, k2, k3);
          if (kb == 7) screen_fast(prev, std::integral_constant<int, 14>{}, std::integral_constant<int, 2>{}, k1, k2, k3);
        }
        // pin the keys to this region (otherwise the IR passes sink the whole
        // screening below the MFMAs, next to its only use)
        asm volatile("" ::"v"(k1), "v"(k2));
      }
      if (!XB && (PCADV_C4_DIAG & 2) == 0 && stg_turn && kb < 4) {  // split the staged f32 rows into bf16 hi / lo, 4 per k-block
#pragma unroll
        for (int j = 4 * kb; j < 4 * kb + 4; ++j) {
          const float v = stg[4 * q + (j >> 2)][j & 3];
          if constexpr (PCADV_C4_CERT >= 2) cert_ss = fmaf(v, v, cert_ss);
          const __bf16 hb = (__bf16)v;
          shi[j >> 3][j & 7] = hb;
          if constexpr (NP4 == 3) slo[j >> 3][j & 7] = (__bf16)(v - (float)hb);
        }
        if (kb == 3) cert_row_done();
        if constexpr (NP4 == 3) asm volatile("" ::"v"(shi[kb >> 1]), "v"(slo[kb >> 1]));
        else asm volatile("" ::"v"(shi[kb >> 1]));
      }
      if ((PCADV_C4_DIAG & 2) == 0 && stg_turn && kb == 4) {  // the next step's tile (buffer free since the barrier)
        bf16x8* dh = reinterpret_cast<bf16x8*>(&L.x[buf ^ 1][0][(srow + 64 * q) * C4_SB + sk]);
        bf16x8* dl = reinterpret_cast<bf16x8*>(&L.x[buf ^ 1][1][(srow + 64 * q) * C4_SB + sk]);
        dh[0] = XB ? stgb[2 * q] : shi[0];
        dh[1] = XB ? stgb[2 * q + 1] : shi[1];
        if constexpr (NP4 == 3) {
          dl[0] = slo[0];
          dl[1] = slo[1];
        }
      }
      // tile s + 2 into the staging registers just freed (clamped: past the
      // end it re-reads the last row): 1.5 units ahead of its conversion
      if ((PCADV_C4_DIAG & 2) == 0 && (G2 || pt == RPT - 1) && kb == 4) stage_load(s + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (decltype(SCREEN)::value) {
      cert_merge(k1, k2, k3);
      pair_merge<NP4 == 3>(k1, uprev, k2, uprev, r1, t1, r2, t2);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if constexpr (G2) {
    // one unit per step (unit 2 s + grp), the previous step's unit screened
    // during it; steps before the last are full, so only the last is masked
    unit(0, grp, accA, accB, F_{}, F_{});
    __syncthreads();
    for (int s = 1; s < S; ++s) {
      if (s & 1) unit(s, grp, accB, accA, T_{}, F_{});
      else unit(s, grp, accA, accB, T_{}, F_{});
      __syncthreads();
    }
  } else if constexpr (P128) {
    // N % 128 == 0: every unit of every step is full, so only the last unit's
    // screen (after the loop) is masked
    unit(0, 0, accA, accB, F_{}, F_{});
    unit(0, 1, accB, accA, T_{}, F_{});
    unit(0, 2, accA, accB, T_{}, F_{});
    unit(0, 3, accB, accA, T_{}, F_{});
    __syncthreads();
    for (int s = 1; s < S; ++s) {
      unit(s, 0, accA, accB, T_{}, F_{});
      unit(s, 1, accB, accA, T_{}, F_{});
      unit(s, 2, accA, accB, T_{}, F_{});
      unit(s, 3, accB, accA, T_{}, F_{});
      __syncthreads();
    }
  } else {
    unit(0, 0, accA, accB, F_{}, F_{});
    if (S > 1) unit(0, 1, accB, accA, T_{}, F_{});
    else unit(0, 1, accB, accA, T_{}, T_{});
    __syncthreads();
    for (int s = 1; s < S; ++s) {
      unit(s, 0, accA, accB, T_{}, F_{});
      if (s + 1 < S) unit(s, 1, accB, accA, T_{}, F_{});
      else unit(s, 1, accB, accA, T_{}, T_{});
      __syncthreads();
#ifdef PCADV_STAMPS
      if ((s & 1) && 6 + (s >> 1) < 14) STAMP(6 + (s >> 1));  // every other step's end
#endif
    }
  }
  // W4 rows of the exact re-evaluation (eight lanes per row, see below): they
  // do not depend on the winners, so they are fetched while the last unit is
  // screened and merged (the W4 fragments' registers are free by now)
  const int oc = lane >> 3, part = lane & 7;
  const float* wbase = w4 + (size_t)(cb * CB + 32 * wblk) * 128 + 16 * part;
  f32x4 wv[4][4];
  if (NP4 == 3 && grp == 0) {
#pragma unroll
    for (int G = 0; G < 4; ++G)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        wv[G][u] = *reinterpret_cast<const f32x4*>(wbase + (size_t)(8 * G + oc) * 128 + 4 * u);
  }
  if constexpr (G2) {  // this wave's last unit
    int k1 = KEY_NONE, k2 = KEY_NONE, k3 = KEY_NONE;
    const int ul = NGRP * (S - 1) + grp;
    if ((S - 1) & 1) screen_unit(accB, ul, T_{}, 0, 8, k1, k2, k3);
    else screen_unit(accA, ul, T_{}, 0, 8, k1, k2, k3);
    cert_merge(k1, k2, k3);
    pair_merge<NP4 == 3>(k1, ul, k2, ul, r1, t1, r2, t2);
  } else {  // the last unit
    int k1 = KEY_NONE, k2 = KEY_NONE, k3 = KEY_NONE;
    screen_unit(accB, UPS * S - 1, T_{}, 0, 8, k1, k2, k3);
    cert_merge(k1, k2, k3);
    pair_merge<NP4 == 3>(k1, UPS * S - 1, k2, UPS * S - 1, r1, t1, r2, t2);
  }
  STAMP(2);

#if PCADV_C4_CERT >= 2
  __shared__ unsigned cert_xn2_wg;  // max over the workgroup's rows (non-negative: uint order)
  if (tid == 0) cert_xn2_wg = 0u;
  __syncthreads();
  atomicMax(&cert_xn2_wg, __float_as_uint(cert_xn2));
  __syncthreads();
  const float cert_xn = sqrtf(__uint_as_float(cert_xn2_wg));
#endif
  // lanes l and l + 32 hold the same channel over interleaved rows
  {
    const int o1 = __shfl_xor(r1, 32), o2 = __shfl_xor(r2, 32);
    // PCADV_C4_CERT: the channel's third screened value = the largest of both
    // lanes' dropped keys and the third of the four candidates merged here
    float cert_v3 = -INFINITY;
    if constexpr (PCADV_C4_CERT && NP4 == 3) {
      const int q3 = max(max(r3, __shfl_xor(r3, 32)),
                         max(min(r1 & ~63, o2 & ~63), min(r2 & ~63, o1 & ~63)));
      cert_v3 = q3 == KEY_NONE ? -INFINITY : key_value(q3);
    }
    const int u1 = __shfl_xor(t1, 32), u2 = __shfl_xor(t2, 32);
    // order by (value, global index): decode both pairs first
    const int hm = 4 * h, ho = 4 - hm;  // row offsets of this lane half and the other
    const int i1 = t1 < 0 ? 0x7fffffff : t1 * 32 + key_row(r1) + hm;
    const int i2 = t2 < 0 ? 0x7fffffff : t2 * 32 + key_row(r2) + hm;
    const int j1 = u1 < 0 ? 0x7fffffff : u1 * 32 + key_row(o1) + ho;
    const int j2 = u2 < 0 ? 0x7fffffff : u2 * 32 + key_row(o2) + ho;
    float v1 = t1 < 0 ? -INFINITY : key_value(r1), v2 = t2 < 0 ? -INFINITY : key_value(r2);
    int a1 = i1, a2 = i2;
    if (ranks_before(v2, a2, v1, a1)) {  // equal truncated values: order by index
      const float tv = v1;
      v1 = v2;
      v2 = tv;
      a1 = i2;
      a2 = i1;
    }
    const float w1v = u1 < 0 ? -INFINITY : key_value(o1), w2v = u2 < 0 ? -INFINITY : key_value(o2);
    // insert (w1v, j1) and (w2v, j2)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float v = q == 0 ? w1v : w2v;
      const int p = q == 0 ? j1 : j2;
      const bool a = ranks_before(v, p, v1, a1);
      const bool b = !a && ranks_before(v, p, v2, a2);
      const float nv2 = a ? v1 : (b ? v : v2);
      const int na2 = a ? a1 : (b ? p : a2);
      v1 = a ? v : v1;
      a1 = a ? p : a1;
      v2 = nv2;
      a2 = na2;
    }
    if constexpr (G2) {  // groups 1.. hand their top-2 of each channel to group 0
      const int slot = 32 * wblk + r;  // lanes r and r + 32 hold the same pair
      // free: the point loop's last barrier has passed (256 slots per group)
      float* xv = L.w[0] + 256 * (grp > 0 ? grp - 1 : 0);
      int* xi = reinterpret_cast<int*>(L.w[1]) + 256 * (grp > 0 ? grp - 1 : 0);
      float* x3v = L.w[2];
      if (grp > 0 && h == 0) {
        xv[2 * slot] = v1;
        xv[2 * slot + 1] = v2;
        xi[2 * slot] = a1;
        xi[2 * slot + 1] = a2;
        if constexpr (PCADV_C4_CERT && NP4 == 3) x3v[slot] = cert_v3;
      }
      __syncthreads();
      if (grp > 0) return;
      if constexpr (PCADV_C4_CERT && NP4 == 3) {
        const float g1 = xv[2 * slot], g2 = xv[2 * slot + 1];
        cert_v3 = fmaxf(fmaxf(cert_v3, x3v[slot]), fmaxf(fminf(v1, g2), fminf(v2, g1)));
      }
#pragma unroll
      for (int q = 0; q < 2 * (NGRP - 1); ++q) {  // group 1's pair, then group 2's, ...
        const float v = xv[256 * (q >> 1) + 2 * slot + (q & 1)];
        const int p = xi[256 * (q >> 1) + 2 * slot + (q & 1)];
        const bool a = ranks_before(v, p, v1, a1);
        const bool b = !a && ranks_before(v, p, v2, a2);
        const float nv2 = a ? v1 : (b ? v : v2);
        const int na2 = a ? a1 : (b ? p : a2);
        v1 = a ? v : v1;
        a1 = a ? p : a1;
        v2 = nv2;
        a2 = na2;
      }
    }
    if (a1 == 0x7fffffff) a1 = 0;
    // The screened top-2 are both re-evaluated as exact f32 dot products and
    // ranked by those values, whatever their screened gap: the screening error
    // (<= ~3 2^-16 sum_k |x_k w_k| from the dropped split products, plus the
    // 2^-17 key truncation) scales with the channel's sum |x w|, which can dwarf
    // a pooled value near 0, so no window on the screened values is safe.  (A
    // third point within the screening error of the top two is not re-checked:
    // DESIGN.md, Numerics.)
    if constexpr (NP4 == 1) {  // bf16 mode: the screened winner and its value
      if (h == 0) {
        float gv = v1 + b4[o];
        int gi = a1;
        if (relu && gv <= 0.f) gv = 0.f, gi = 0;  // see below
        gmax[(size_t)c * C4_O + o] = gv;
        gidx[(size_t)c * C4_O + o] = gi;
      }
      return;
    }
    const bool near = a2 != 0x7fffffff;
    const int b2 = near ? a2 : a1;
    STAMP(4);
    // Exact dot products, eight lanes per row: in pass G lane l takes channel
    // 8 G + (l >> 3) and terms 16 (l & 7) .. + 16, so a load instruction reads
    // eight 128-B lines whole (a lane-per-row layout would touch 64 lines) and
    // the partial sums meet in three DPP steps within the lane octet.
    f32x4 av[4][4], bv[4][4];
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      const int ch = 8 * G + oc;
      const int p1 = __shfl(a1, ch), p2 = __shfl(b2, ch);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[G][u] = *reinterpret_cast<const f32x4*>(xc + (size_t)p1 * 128 + 16 * part + 4 * u);
        bv[G][u] = *reinterpret_cast<const f32x4*>(xc + (size_t)p2 * 128 + 16 * part + 4 * u);
      }
    }
#ifdef PCADV_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
#endif
    STAMP(5);
    float res1 = 0.f, res2 = 0.f;
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      float e1 = 0.f, e2 = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          e1 = fmaf(av[G][u][t], wv[G][u][t], e1);
          e2 = fmaf(bv[G][u][t], wv[G][u][t], e2);
        }
      e1 = octet_sum(e1);
      e2 = octet_sum(e2);
      // channel ch = 8 G + k was summed in lanes 8 k .. 8 k + 7: owner lanes
      // r in [8 G, 8 G + 8) (both halves) fetch it
      const int src = 8 * ((r - 8 * G) & 7);
      const float f1 = __shfl(e1, src), f2 = __shfl(e2, src);
      if ((r >> 3) == G) {
        res1 = f1;
        res2 = f2;
      }
    }
    const float bias = b4[o];
    const float e1 = res1 + bias, e2 = res2 + bias;
    const bool second = near && ranks_before(e2, a2, e1, a1);
    if (h == 0) {
      float gv = second ? e2 : e1;
      int gi = second ? a2 : a1;
      // relu (the T-Nets' ReLU before the max, pointnet.py:30-31,63-64):
      // max_n relu(v) = relu(max_n v), and where every v <= 0 the ReLU'd row
      // is all zeros, whose first index (torch.max) is point 0
      if (relu && gv <= 0.f) gv = 0.f, gi = 0;
      gmax[(size_t)c * C4_O + o] = gv;
      gidx[(size_t)c * C4_O + o] = gi;
    }
#if PCADV_C4_CERT == 1
    asm volatile("" ::"v"(cert_v3));  // tracking cost only
#elif PCADV_C4_CERT >= 2
    {
      // a dropped point p has exact value <= s_p + err_p <= v3 + err, with the
      // screening error err <= 2^-14.3 sum_k |x_pk w_ok| (three dropped split
      // terms <= 3 2^-18, up to 384 f32 accumulation roundings <= 2^-15.4, the
      // 2^-17 key truncation) <= 2^-14 ||x_p|| ||w_o|| (Cauchy-Schwarz)
      float wn2 = 0.f;
      for (int k = 0; k < 128; ++k) wn2 = fmaf(w4[(size_t)o * 128 + k], w4[(size_t)o * 128 + k], wn2);
      const float bound = cert_xn * sqrtf(wn2);
      const float ew = second ? res2 : res1;  // the winner's exact value, no bias
      if (h == 0) {
        atomicAdd(&g_c4_cert[0], cert_v3 + 0x1p-14f * bound >= ew ? 1u : 0u);
        atomicAdd(&g_c4_cert[1], 1u);
        atomicAdd(&g_c4_cert[2], cert_v3 + 0x1p-17f * bound >= ew ? 1u : 0u);
      }
      if (blockIdx.x == 0 && tid == 0) atomicAdd(&g_c4_cert[3], 1u);
    }
#endif
  }
  STAMP(3);
#undef STAMP
}

#if PCADV_C4_CERT
// diagnostic builds only: read (and reset) the certification counters
int c4_cert_read(unsigned* host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_c4_cert), sizeof(g_c4_cert)) != hipSuccess) return -1;
  const unsigned z[4] = {0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_c4_cert), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

size_t feat_fwd_workspace_bytes(int C, int N) {
  (void)C;
  (void)N;
  return 256;  // no scratch: kept so callers can size a shared workspace
}

template <int NP3, int NP4>
static int feat_fwd_attrs() {
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_conv4_max<NP4, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(C4Lds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_conv4_max<NP4, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(C4Lds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_conv4_max<NP4, false, NP4 == 1>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(C4Lds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_conv4_max<NP4, true, NP4 == 1>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(C4Lds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_conv4_max<NP4, false, false, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(C4Lds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_conv4_max<NP4, false, NP4 == 1, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(C4Lds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_point_mlp<NP3, 2, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(MlpLds<2, false>)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_point_mlp<NP3, 1, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(MlpLds<1, false>)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_point_mlp<NP3, 2, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(MlpLds<2, true>)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_point_mlp<NP3, 1, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(MlpLds<1, true>)) != hipSuccess) {
      set_error("feat_fwd: cannot reserve LDS (%zu / %zu bytes)", sizeof(C4Lds), sizeof(MlpLds<2, false>));
      return PCADV_EHIP;
    }
    attr_set = true;
  }
  return PCADV_OK;
}

// k_conv4_max alone over a given x3 (C x N x 128): the second launch of the
// feature forward.  XB: x3 is bf16 (bf16 mode's k_point_mlp store)
template <int NP3, int NP4, bool XB = false>
static int launch_conv4_max_np(const float* x3, int C, int N, const float* w4, const float* b4,
                               float* gmax, int32_t* gidx, hipStream_t s, uint64_t* stamps,
                               int relu = 0) {
  const int rc = feat_fwd_attrs<NP3, NP4>();
  if (rc != PCADV_OK) return rc;
  // two wave groups per 128-channel workgroup when 256-channel workgroups would
  // leave CUs idle (the diagnostic stamps layout assumes the plain form)
#ifndef PCADV_C4_G2_MAXC
#define PCADV_C4_G2_MAXC 63  // A/B builds: the largest cloud count run in the two-group form
#endif
  if (C <= PCADV_C4_G2_MAXC && !stamps)
    hipLaunchKernelGGL((k_conv4_max<NP4, true, XB>), dim3(C * (2 * C4_O / C4_CB)),
                       dim3(c4_threads<NP4, true, XB>()),
                       sizeof(C4Lds), s, x3, C, N, w4, b4, gmax, gidx, stamps, relu);
  else if (PCADV_C4_P128 && N % 128 == 0 && !stamps)
    hipLaunchKernelGGL((k_conv4_max<NP4, false, XB, true>), dim3(C * (C4_O / C4_CB)), dim3(C4_T),
                       sizeof(C4Lds), s, x3, C, N, w4, b4, gmax, gidx, stamps, relu);
  else
    hipLaunchKernelGGL((k_conv4_max<NP4, false, XB>), dim3(C * (C4_O / C4_CB)), dim3(C4_T),
                       sizeof(C4Lds), s, x3, C, N, w4, b4, gmax, gidx, stamps, relu);
  PC_HIP_CHECK_LAUNCH("k_conv4_max");
  return PCADV_OK;
}

template <int NP3, int NP4>
static int launch_feat_fwd_np(const float* pts_a, const float* pts_b, int split, int C, int N,
                              const float* w1, const float* b1, const float* w2, const float* b2,
                              const float* w3, const float* b3, const float* w4, const float* b4,
                              float* x3, float* gmax, int32_t* gidx, int32_t* inc_counter,
                              hipStream_t s, uint64_t* stamps, const GatherFold& gf) {
  const int rc = feat_fwd_attrs<NP3, NP4>();
  if (rc != PCADV_OK) return rc;
  const int T = (N + PM_P - 1) / PM_P;
  const int ntiles = C * T;
  uint64_t* mlp_stamps = stamps ? stamps + (size_t)C * (C4_O / C4_CB) * 16 : nullptr;
  // one tile per workgroup when two would give fewer than two workgroups per
  // CU (512); the diagnostic stamps layout assumes two
#ifndef PCADV_MLP_ONE_BELOW
#define PCADV_MLP_ONE_BELOW 1024  // A/B builds: the tile count below which one tile per workgroup runs
#endif
  const bool one = ntiles < PCADV_MLP_ONE_BELOW && !stamps;
  const dim3 grid(one ? ntiles : (ntiles + 1) / 2);
  auto kern = one ? (gf.n ? k_point_mlp<NP3, 1, true> : k_point_mlp<NP3, 1, false>)
                  : (gf.n ? k_point_mlp<NP3, 2, true> : k_point_mlp<NP3, 2, false>);
  const size_t lds = one ? sizeof(MlpLds<1, false>) : gf.n ? sizeof(MlpLds<2, true>) : sizeof(MlpLds<2, false>);
  hipLaunchKernelGGL(kern, grid, dim3(PM_T), lds, s, pts_a, pts_b, split, N, T, ntiles,
                     w1, b1, w2, b2, w3, b3, x3, inc_counter, mlp_stamps, gf);
  PC_HIP_CHECK_LAUNCH("k_point_mlp");
  // bf16 mode: k_point_mlp<1> stored x3 as bf16
  return launch_conv4_max_np<NP3, NP4, NP3 == 1>(x3, C, N, w4, b4, gmax, gidx, s, stamps);
}

int launch_conv4_max(const float* x3, int C, int N, const float* w4, const float* b4, float* gmax,
                     int32_t* gidx, hipStream_t s, int precision, int relu) {
  PC_REQUIRE(C > 0 && N > 0, "conv4_max: bad shape C=%d N=%d", C, N);
  PC_REQUIRE(precision >= 0 && precision <= 2,
             "conv4_max: precision %d (0 fp32, 1 bf16, 2 bf16 over a bf16 x3)", precision);
  if (precision == 2)
    return launch_conv4_max_np<1, 1, true>(x3, C, N, w4, b4, gmax, gidx, s, nullptr, relu);
  if (precision == 1)
    return launch_conv4_max_np<1, 1>(x3, C, N, w4, b4, gmax, gidx, s, nullptr, relu);
  return launch_conv4_max_np<6, 3>(x3, C, N, w4, b4, gmax, gidx, s, nullptr, relu);
}

// precision 0: f32-level (conv3 six bf16 products, conv4 three + the exact
// re-evaluation); 1: bf16 (one product each, the screened winner as is)
int launch_feat_fwd_fused(const float* pts_a, const float* pts_b, int split, int C, int N,
                          const float* w1, const float* b1, const float* w2, const float* b2,
                          const float* w3, const float* b3, const float* w4, const float* b4,
                          float* x3, float* gmax, int32_t* gidx, int32_t* inc_counter, void* ws,
                          size_t ws_bytes, hipStream_t s, uint64_t* stamps, int precision,
                          const pcadv_gather_job* gather, int ngather) {
  (void)ws;
  (void)ws_bytes;
  PC_REQUIRE(C > 0 && N > 0, "feat_fwd: bad shape C=%d N=%d", C, N);
  PC_REQUIRE((size_t)C * 4 <= 0x7fffffff / 1, "feat_fwd: too many clouds (%d)", C);
  PC_REQUIRE(precision == 0 || precision == 1, "feat_fwd: precision %d (0 fp32, 1 bf16)", precision);
  GatherFold gf{};
  if (ngather) {
    // job 0 fills clouds [0, split) from pts_a, job 1 clouds [split, C) from pts_b
    const int want = split < C ? 2 : 1;
    PC_REQUIRE(gather && ngather == want, "feat_fwd: %d gather jobs for this batch (want %d)",
               ngather, want);
    for (int k = 0; k < ngather; ++k) {
      const pcadv_gather_job& j = gather[k];
      const float* pts = k == 0 ? pts_a : pts_b;
      const int rows = k == 0 ? split : C - split;
      PC_REQUIRE(j.src && j.order && j.cursor && j.out == pts && j.B == rows && j.npts == N &&
                     j.src_npts >= N && j.n_src > 0,
                 "feat_fwd: gather job %d does not fill its %d x %d input batch", k, rows, N);
      PC_REQUIRE(j.sigma >= 0.0 && (j.sigma == 0.0 || j.clip > 0.0),
                 "feat_fwd: gather job %d: clip must be > 0", k);
      PC_REQUIRE(!j.src_lab || (j.lab_width > 0 && j.lab_width <= N && j.out_lab),
                 "feat_fwd: gather job %d: labels", k);
      PC_REQUIRE(!j.src_seg, "feat_fwd: gather job %d: part ids are not gathered here", k);
      gf.j[k] = j;
    }
    gf.n = ngather;
  }
  if (precision == 1)
    return launch_feat_fwd_np<1, 1>(pts_a, pts_b, split, C, N, w1, b1, w2, b2, w3, b3, w4, b4, x3,
                                    gmax, gidx, inc_counter, s, stamps, gf);
  return launch_feat_fwd_np<6, 3>(pts_a, pts_b, split, C, N, w1, b1, w2, b2, w3, b3, w4, b4, x3,
                                  gmax, gidx, inc_counter, s, stamps, gf);
}

}  // namespace pcadv

// Fused PointNetfeat forward (models/pointnet.py:109-132, feature_transform=False)
// on gfx950: conv1 -> conv2 -> conv3 -> conv4 -> max over points, one
// workgroup per (cloud, 128-point tile), nothing but conv3's output leaves the
// chip.
//
//   conv1 (3 -> 64)    VALU, exact f32
//   conv2 (64 -> 64)   v_mfma_f32_32x32x2_f32 (exact f32)
//   conv3 (64 -> 128)  v_mfma_f32_32x32x2_f32; x3 is written to HBM in f32 (the
//                      backward and the exact re-evaluation below read it) and
//                      kept in LDS split as bf16 hi + lo
//   conv4 (128 -> 1024) + max: three bf16 MFMAs per product
//                      (x_hi w_hi + x_hi w_lo + x_lo w_hi, f32 accumulate,
//                      v_mfma_f32_32x32x16_bf16): relative error <= ~1.2e-5 of
//                      sum|x w|, at 16x the per-cycle rate of the f32 MFMA.  The
//                      epilogue keeps the top-2 (value, point) per channel.
//
// k_gmax_combine then merges the per-tile top-2 keys of each channel and
// re-evaluates the winner in exact f32 (and the runner-up whenever the two are
// within the split-product error bound), so gmax is an f32 dot product and the
// argmax follows the f32 values, first index on ties (torch.max on CPU).
#include "common.h"

namespace pcadv {

constexpr int FF_P = 128;   // points per workgroup
constexpr int FF_T = 1024;  // threads (16 waves = 4 per SIMD, 1 workgroup per CU)
constexpr int FF_SB = 136;  // bf16 row stride of the x3 hi/lo tiles (272 B)
constexpr int FF_O = 1024;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Two 128-point tiles per workgroup.  X holds tile A's conv3 output split to
// bf16 hi/lo; Y holds tile A's, then tile B's conv1/conv2 outputs (f32), and
// finally tile B's split conv3 output.
struct FwdLds {
  alignas(16) float pts[2][FF_P * 4];
  alignas(16) __bf16 x[2][FF_P * FF_SB];  // tile A x3: hi, lo
  union U {
    struct {
      float x1[FF_P * S64];
      float x2[FF_P * S64];
    } f;
    __bf16 x3[2][FF_P * FF_SB];            // tile B x3: hi, lo
  };
  alignas(16) U y;
  int sync[2];                             // producer-wave arrival counters
};

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Screening keys: the f32 value mapped to an order-preserving int32 with the
// point's index inside the 128-point tile packed into the low 7 bits (stored
// as 127 - idx, so equal screening values rank the lower index first).  One
// v_max_i32 + one v_med3_i32 then keep the top-2 (value, point) pairs; the 7
// dropped mantissa bits (2^-16 relative) sit far inside the near-tie window
// that k_gmax_combine re-checks in exact f32.
__device__ __forceinline__ int screen_key(float v, int idx) {
  const int b = __float_as_int(v);
  const int ord = b ^ ((b >> 31) & 0x7fffffff);   // int order == float order
  return (ord & ~0x7f) | (127 - idx);
}
__device__ __forceinline__ float key_value(int k) {
  const int ord = k & ~0x7f;
  return __int_as_float(ord ^ ((ord >> 31) & 0x7fffffff));
}
__device__ __forceinline__ int key_index(int k) { return 127 - (k & 0x7f); }
constexpr int KEY_NONE = (int)0x80000000;  // below every real key

__device__ __forceinline__ void key_push(int k, int& k1, int& k2) {
  k2 = max(min(k, k1), k2);  // median(k, k1, k2) for k2 <= k1: v_med3_i32
  k1 = max(k1, k);
}

// (va, ia) ranks before (vb, ib): larger value, NaN above all, lower index on ties
__device__ __forceinline__ bool ranks_before(float va, int ia, float vb, int ib) {
  const bool na = va != va, nb = vb != vb;
  if (na || nb) return na && (!nb || ia < ib);
  return va > vb || (va == vb && ia < ib);
}

__device__ __forceinline__ void top2_merge(float v, int p, float& v1, int& i1, float& v2, int& i2) {
  const bool a = ranks_before(v, p, v1, i1);
  const bool b = !a && ranks_before(v, p, v2, i2);
  const float nv2 = a ? v1 : (b ? v : v2);
  const int ni2 = a ? i1 : (b ? p : i2);
  v1 = a ? v : v1;
  i1 = a ? p : i1;
  v2 = nv2;
  i2 = ni2;
}

// wave-group barrier among the 4 producer waves (4..7) through an LDS counter:
// every wave publishes its LDS writes, then waits for the others
// (every spin is bounded: a lost arrival cannot hang the device)
__device__ __forceinline__ void group_wait(int* cnt, int target) {
  for (int spin = 0; spin < (1 << 22); ++spin) {
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void group_sync(int* cnt, int target) {
  __builtin_amdgcn_s_waitcnt(0);  // this wave's LDS (and memory) writes are done
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  group_wait(cnt, target);
}

// conv4 weights split once per launch into bf16 hi / lo ([1024][128] each), so
// the screening loop loads its B operands directly
__global__ void __launch_bounds__(256)
k_w4_split(const float* __restrict__ w4, __bf16* __restrict__ hi, __bf16* __restrict__ lo) {
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= FF_O * 128) return;
  const f32x4 v = *reinterpret_cast<const f32x4*>(w4 + i);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 hb = (__bf16)v[j];
    hi[i + j] = hb;
    lo[i + j] = (__bf16)(v[j] - (float)hb);
  }
}

constexpr int FF_NB = 2;   // tile-A units a consumer wave runs while tile B's conv1-3 run
constexpr int FF_NCW = 8;  // consumer waves (0-7); producer waves 8-15

// Pipelined over two point tiles A, B of one cloud (16 waves, 4 per SIMD):
//   phase A  all waves: conv1..conv3 of tile A (x1, x2 in Y; x3 -> HBM + X)
//   phase B  waves 0-7: conv4 + screening of tile A, 2 of their 4 channel
//            units; waves 8-15: conv1..conv3 of tile B (x3 kept in registers)
//   phase C  waves 8-15 split tile B's x3 into Y; waves 0-7 finish their 2
//            tile-A units and take 1 tile-B unit each, waves 8-15 take 3
//            tile-B units each (32 tile-B units in all)
// A unit is 32 channels x 128 points, run in two 64-point halves so that a
// wave stays within 128 VGPRs: four waves per SIMD keep the matrix pipe fed
// while any one of them waits on LDS or runs its screening epilogue.
__global__ void __launch_bounds__(FF_T)
k_feat_fwd_fused(const float* __restrict__ pts_a, const float* __restrict__ pts_b, int split,
                 int N, const float* __restrict__ w1, const float* __restrict__ b1,
                 const float* __restrict__ w2, const float* __restrict__ b2,
                 const float* __restrict__ w3, const float* __restrict__ b3,
                 const __bf16* __restrict__ w4hi, const __bf16* __restrict__ w4lo,
                 float* __restrict__ x3g, int2* __restrict__ part, int32_t* inc_counter,
                 uint64_t* __restrict__ stamps, int T) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  FwdLds& L = *reinterpret_cast<FwdLds*>(smem);
#ifdef PCADV_STAMPS
  // diagnostic build only: per-workgroup phase timestamps (s_memrealtime, 100 MHz)
  uint64_t* st = stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16;
#define STAMP(k) do { if (stamps && (threadIdx.x & 63) == 0) st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP(k) do { } while (0)
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int c = blockIdx.y, tA = 2 * blockIdx.x, tB = tA + 1;
  const bool hasB = tB < T;
  if (wave == 0) STAMP(0);
  if (inc_counter && tid == 0 && c == 0 && blockIdx.x == 0) *inc_counter += 1;
  const float* pts = c < split ? pts_a + (size_t)c * N * 3 : pts_b + (size_t)(c - split) * N * 3;

  for (int e = tid; e < 2 * FF_P * 3; e += FF_T) {
    const int t = e / (FF_P * 3), p = (e % (FF_P * 3)) / 3, k = e % 3;
    const int gp = (tA + t) * FF_P + p;
    L.pts[t][p * 4 + k] = gp < N ? pts[(size_t)gp * 3 + k] : 0.f;
  }
  if (tid < 2) L.sync[tid] = 0;
  __syncthreads();

  // ---- conv1 (3 -> 64) + ReLU of one tile: NT threads = (channel, point group)
  auto conv1 = [&](const float* ps, int t0, int NT) {
    const int ch = t0 & 63, pg = t0 >> 6, per = FF_P / (NT / 64);
    const float wa = w1[ch * 3 + 0], wb = w1[ch * 3 + 1], wc = w1[ch * 3 + 2], bb = b1[ch];
    for (int i = 0; i < per; ++i) {
      const int p = pg * per + i;
      L.y.f.x1[p * S64 + ch] = conv1_point(wa, wb, wc, bb, ps[p * 4 + 0], ps[p * 4 + 1], ps[p * 4 + 2]);
    }
  };
  // ---- conv2 (64 -> 64) + ReLU, one 32x32 tile (point tile pt, channel tile ct)
  auto conv2 = [&](int pt, int ct) {
    f32x4 bf[8];
    load_bfrag<64>(w2, 32 * ct, lane, bf);
    f32x16 acc = {};
    acc = mfma_rows_x_wt<64>(L.y.f.x1 + 32 * pt * S64, S64, bf, acc, lane);
    const int col = 32 * ct + r;
    const float bias = b2[col];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[i] + bias;
      L.y.f.x2[(32 * pt + acc_row(i, lane)) * S64 + col] = v > 0.f ? v : 0.f;
    }
  };
  // ---- conv3 (64 -> 128) + ReLU, one 32x32 tile; the value also goes to HBM
  auto conv3 = [&](int tile, int pt, int ct, f32x16& acc) {
    f32x4 bf[8];
    load_bfrag<64>(w3, 32 * ct, lane, bf);
    acc = f32x16{};
    acc = mfma_rows_x_wt<64>(L.y.f.x2 + 32 * pt * S64, S64, bf, acc, lane);
    const int col = 32 * ct + r;
    const float bias = b3[col];
    const int p0 = tile * FF_P;
    float* xg = x3g + ((size_t)c * N + p0) * 128 + col;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = 32 * pt + acc_row(i, lane);
      float v = acc[i] + bias;
      v = v > 0.f ? v : 0.f;
      acc[i] = v;
      if (p0 + row < N) xg[(size_t)row * 128] = v;
    }
  };
  auto x3_split = [&](__bf16* hi, __bf16* lo, int pt, int ct, const f32x16& acc) {
    const int col = 32 * ct + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = 32 * pt + acc_row(i, lane);
      const __bf16 hb = (__bf16)acc[i];
      hi[row * FF_SB + col] = hb;
      lo[row * FF_SB + col] = (__bf16)(acc[i] - (float)hb);
    }
  };

  // ================= phase A: conv1..conv3 of tile A, all waves ===============
  conv1(L.pts[0], tid, FF_T);
  __syncthreads();
  if (wave < 8) conv2(wave >> 1, wave & 1);
  __syncthreads();
  {
    f32x16 acc;
    conv3(tA, wave >> 2, wave & 3, acc);
    x3_split(L.x[0], L.x[1], wave >> 2, wave & 3, acc);
  }
  __syncthreads();
  if (wave == 0 || wave == 8) STAMP(1 + (wave >> 3));

  // ---- conv4 (128 -> 1024) split-bf16 MFMA + top-2 screening of one channel
  //      unit (32 channels x the tile's 128 points) --------------------------
  auto conv4_unit = [&](const __bf16* xhi, const __bf16* xlo, int tile, int ct) {
    const int p0 = tile * FF_P;
    const bool full = p0 + FF_P <= N;
    const int o0 = 32 * ct;
    // B operands: lane (r, h) holds W4[o0 + r][16 kb + 8 h .. + 8) hi and lo
    bf16x8 bh[8], bl[8];
    {
      const __bf16* ph = w4hi + (size_t)(o0 + r) * 128 + 8 * h;
      const __bf16* pl = w4lo + (size_t)(o0 + r) * 128 + 8 * h;
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        bh[kb] = *reinterpret_cast<const bf16x8*>(ph + 16 * kb);
        bl[kb] = *reinterpret_cast<const bf16x8*>(pl + 16 * kb);
      }
    }
    int k1 = KEY_NONE, k2 = KEY_NONE;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const __bf16* xh = xhi + (64 * half + r) * FF_SB + 8 * h;
      const __bf16* xl = xlo + (64 * half + r) * FF_SB + 8 * h;
      f32x16 acc[2] = {{}, {}};
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        // bound the scheduler's look-ahead to one k-block: within 128 VGPRs the
        // other three waves of the SIMD, not deep prefetch, hide LDS latency
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const bf16x8 ah = *reinterpret_cast<const bf16x8*>(xh + 32 * pt * FF_SB + 16 * kb);
          const bf16x8 al = *reinterpret_cast<const bf16x8*>(xl + 32 * pt * FF_SB + 16 * kb);
          acc[pt] = mfma_bf16(al, bh[kb], acc[pt]);
          acc[pt] = mfma_bf16(ah, bl[kb], acc[pt]);
          acc[pt] = mfma_bf16(ah, bh[kb], acc[pt]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // screening top-2 over these 64 points (bias is added by the exact
      // re-evaluation in k_gmax_combine; it does not change the order)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int idx = 64 * half + 32 * pt + acc_row(i, lane);
          if (full || p0 + idx < N) key_push(screen_key(acc[pt][i], idx), k1, k2);
        }
    }
    // lanes l and l+32 hold the same channel over interleaved rows
    const int o1 = __shfl_xor(k1, 32), o2 = __shfl_xor(k2, 32);
    k2 = max(min(k1, o1), max(k2, o2));
    k1 = max(k1, o1);
    if (lane < 32) part[((size_t)c * T + tile) * FF_O + o0 + r] = make_int2(k1, k2);
  };

  // unit lists: consumer wave w (0-7) owns tile-A channel tiles 4w..4w+3;
  // tile-B channel tiles: producers (8-15) -> 3 each from 0, consumers -> 1 each from 24
  const bool consumer = wave < FF_NCW;
  const int nBu = hasB ? (consumer ? 1 : 3) : 0;
  const int bBase = consumer ? 24 + wave : 3 * (wave - FF_NCW);

  if (consumer) {
    // ================= phase B, consumers: tile-A units 0..FF_NB-1 ===========
    for (int j = 0; j < FF_NB; ++j) conv4_unit(L.x[0], L.x[1], tA, 4 * wave + j);
    STAMP(3);
  } else if (hasB) {
    // ================= phase B, producers: conv1..conv3 of tile B =============
    const int pw = wave - FF_NCW;
    conv1(L.pts[1], tid - 64 * FF_NCW, FF_T - 64 * FF_NCW);
    group_sync(&L.sync[0], 8);
    conv2(pw >> 1, pw & 1);
    group_sync(&L.sync[0], 16);
    f32x16 acc3[2];
    conv3(tB, pw >> 2, pw & 3, acc3[0]);
    conv3(tB, (pw >> 2) + 2, pw & 3, acc3[1]);
    STAMP(4);
    // ================= phase C, producers: split tile B's x3 into Y ===========
    group_sync(&L.sync[1], 8);  // every producer's conv3 MFMAs have read x2
    x3_split(L.y.x3[0], L.y.x3[1], pw >> 2, pw & 3, acc3[0]);
    x3_split(L.y.x3[0], L.y.x3[1], (pw >> 2) + 2, pw & 3, acc3[1]);
    group_sync(&L.sync[1], 16);
  }

  if (consumer) {
    // ================= phase C, consumers: remaining tile-A units =============
    for (int j = FF_NB; j < 4; ++j) conv4_unit(L.x[0], L.x[1], tA, 4 * wave + j);
    if (nBu > 0) group_wait(&L.sync[1], 16);  // tile B's split x3 is complete
  }
  for (int j = 0; j < nBu; ++j) conv4_unit(L.y.x3[0], L.y.x3[1], tB, bBase + j);
  if (wave == 0 || wave == 8) STAMP(5 + (wave >> 3));
#undef STAMP
}

// Four lanes per (cloud, channel): merge the T tile partials (top-2 screening
// keys), then exact f32 dot products over x3 rows (each lane 32 of the 128
// terms) for the winner and, on near-ties, the runner-up.
__global__ void __launch_bounds__(256)
k_gmax_combine(const int2* __restrict__ part, int T, int C, int N,
               const float* __restrict__ x3g, const float* __restrict__ w4,
               const float* __restrict__ b4, float* __restrict__ gmax,
               int32_t* __restrict__ gidx) {
  const int q = threadIdx.x & 3;
  const int g = blockIdx.x * 64 + (threadIdx.x >> 2);  // (cloud, channel) pair
  const int c = g / FF_O, o = g % FF_O;
  if (c >= C) return;  // C * FF_O is a multiple of 64: whole waves leave
  // this lane's quarter of W4[o] and the bias do not depend on the merge:
  // fetched together with the partials
  const float* wrow = w4 + (size_t)o * 128 + 32 * q;
  f32x4 wv[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) wv[u] = *reinterpret_cast<const f32x4*>(wrow + 4 * u);
  const float bias = b4[o];
  float v1 = -INFINITY, v2 = -INFINITY;
  int i1 = 0x7fffffff, i2 = 0x7fffffff;
  for (int t = q; t < T; t += 4) {
    const int2 kk = part[((size_t)c * T + t) * FF_O + o];
    if (kk.x != KEY_NONE) top2_merge(key_value(kk.x), t * FF_P + key_index(kk.x), v1, i1, v2, i2);
    if (kk.y != KEY_NONE) top2_merge(key_value(kk.y), t * FF_P + key_index(kk.y), v1, i1, v2, i2);
  }
#pragma unroll
  for (int m = 1; m < 4; m <<= 1) {
    const float a1 = __shfl_xor(v1, m), a2 = __shfl_xor(v2, m);
    const int j1 = __shfl_xor(i1, m), j2 = __shfl_xor(i2, m);
    top2_merge(a1, j1, v1, i1, v2, i2);
    top2_merge(a2, j2, v1, i1, v2, i2);
  }
  if (i1 == 0x7fffffff) i1 = 0;
  // screening error <= ~1.2e-5 sum|x w| (+2^-16 key truncation): re-check
  // anything within a far wider window of the winner in exact f32; both rows
  // are fetched in one round trip
  const bool near = i2 != 0x7fffffff && !(v1 - v2 > 1e-3f * (fabsf(v1) + fabsf(v2)) + 1e-6f);
  const float* x1r = x3g + ((size_t)c * N + i1) * 128 + 32 * q;
  const float* x2r = x3g + ((size_t)c * N + (near ? i2 : i1)) * 128 + 32 * q;
  f32x4 xa[8], xb[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) xa[u] = *reinterpret_cast<const f32x4*>(x1r + 4 * u);
  if (near) {
#pragma unroll
    for (int u = 0; u < 8; ++u) xb[u] = *reinterpret_cast<const f32x4*>(x2r + 4 * u);
  }
  auto dot = [&](const f32x4* xv) {
    float d = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      d = fmaf(xv[u].x, wv[u].x, d);
      d = fmaf(xv[u].y, wv[u].y, d);
      d = fmaf(xv[u].z, wv[u].z, d);
      d = fmaf(xv[u].w, wv[u].w, d);
    }
    d += __shfl_xor(d, 1);
    d += __shfl_xor(d, 2);
    return d;
  };
  const float e1 = dot(xa) + bias;
  float e2 = 0.f;
  if (near) e2 = dot(xb) + bias;
  const bool second = near && ranks_before(e2, i2, e1, i1);
  if (q == 0) {
    gmax[(size_t)c * FF_O + o] = second ? e2 : e1;
    gidx[(size_t)c * FF_O + o] = second ? i2 : i1;
  }
}

// workspace: per-tile top-2 partials, then W4 split into bf16 hi / lo
static size_t part_bytes(int C, int N) {
  const size_t T = (N + FF_P - 1) / FF_P;
  return ((size_t)C * T * FF_O * sizeof(int2) + 255) & ~(size_t)255;
}

size_t feat_fwd_workspace_bytes(int C, int N) {
  return part_bytes(C, N) + 2 * (size_t)FF_O * 128 * sizeof(__bf16);
}

int launch_feat_fwd_fused(const float* pts_a, const float* pts_b, int split, int C, int N,
                          const float* w1, const float* b1, const float* w2, const float* b2,
                          const float* w3, const float* b3, const float* w4, const float* b4,
                          float* x3, float* gmax, int32_t* gidx, int32_t* inc_counter, void* ws,
                          size_t ws_bytes, hipStream_t s, uint64_t* stamps) {
  PC_REQUIRE(C > 0 && N > 0, "feat_fwd: bad shape C=%d N=%d", C, N);
  PC_REQUIRE(ws && ws_bytes >= feat_fwd_workspace_bytes(C, N), "feat_fwd: workspace too small");
  const int T = (N + FF_P - 1) / FF_P;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_feat_fwd_fused),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(FwdLds)) != hipSuccess) {
      set_error("feat_fwd: cannot reserve %zu bytes of LDS", sizeof(FwdLds));
      return PCADV_EHIP;
    }
    attr_set = true;
  }
  int2* part = static_cast<int2*>(ws);
  __bf16* w4hi = reinterpret_cast<__bf16*>(static_cast<char*>(ws) + part_bytes(C, N));
  __bf16* w4lo = w4hi + FF_O * 128;
  hipLaunchKernelGGL(k_w4_split, dim3(FF_O * 128 / 4 / 256), dim3(256), 0, s, w4, w4hi, w4lo);
  PC_HIP_CHECK_LAUNCH("k_w4_split");
  hipLaunchKernelGGL(k_feat_fwd_fused, dim3((T + 1) / 2, C), dim3(FF_T), sizeof(FwdLds), s, pts_a,
                     pts_b, split, N, w1, b1, w2, b2, w3, b3, w4hi, w4lo, x3, part, inc_counter,
                     stamps, T);
  PC_HIP_CHECK_LAUNCH("k_feat_fwd_fused");
  hipLaunchKernelGGL(k_gmax_combine, dim3(C * FF_O / 64), dim3(256), 0, s, part, T, C, N, x3, w4,
                     b4, gmax, gidx);
  PC_HIP_CHECK_LAUNCH("k_gmax_combine");
  return PCADV_OK;
}

}  // namespace pcadv

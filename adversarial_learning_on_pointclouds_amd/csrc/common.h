// Shared helpers for the pcadv HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

#include "../../include/pcadv.h"

namespace pcadv {

// thread-local last-error text (pcadv_last_error)
void set_error(const char* fmt, ...);

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// f32 -> three bf16 whose sum is the f32 value (round-to-nearest splits: each
// residual is exact in f32 and the last one fits 8 significant bits).  Six
// products of two such splits (l h, m m, h l, m h, h m, h h; the dropped terms
// are < 2^-23 of |a b|) give an f32-level product on the bf16 matrix pipe.
__device__ __forceinline__ void split3(float v, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)v;
  const float r1 = v - (float)hi;
  mid = (__bf16)r1;
  lo = (__bf16)(r1 - (float)mid);
}

// 32x32x2 f32 MFMA: exact f32 (k-ordered fma chain), 64 cycles / SIMD.
// lane l supplies A[i=l&31][k=l>>5], B[k=l>>5][j=l&31];
// D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

// Kernel arguments are read by scalar loads at their first use, and a use that
// sits behind a branch on another argument costs a further dependent round trip
// to the kernarg segment (0.6-0.8 us each at the start of a launch, measured by
// tools/lin_stamps.py).  Naming every argument a kernel reads at its entry lets
// the compiler issue all of those loads together: one round trip.
template <typename T>
__device__ __forceinline__ void kernarg_pin(const T& v) {
  asm volatile("" ::"s"(v));
}
template <typename... T>
__device__ __forceinline__ void kernarg_prefetch(const T&... v) {
  (kernarg_pin(v), ...);
}

// activation codes shared with the C ABI (include/pcadv.h)
enum Act { ACT_NONE = PCADV_ACT_NONE, ACT_RELU = PCADV_ACT_RELU, ACT_LRELU = PCADV_ACT_LRELU };

__device__ __forceinline__ float act_fwd(float x, int act) {
  if (act == ACT_RELU) return x > 0.f ? x : 0.f;
  if (act == ACT_LRELU) return x > 0.f ? x : x * 0.2f;
  return x;
}
// derivative from the activation OUTPUT (sign preserved by relu/leaky relu)
__device__ __forceinline__ float act_bwd(float y, int act) {
  if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == ACT_LRELU) return y > 0.f ? 1.f : 0.2f;
  return 1.f;
}

// ---------------------------------------------------------------------------
// counter-based RNG (Philox-4x32-10) for dropout masks and soft D labels.
// Keyed by (seed, step counter read on device) so graph replays draw fresh
// numbers each step without host involvement.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  return {c0, c1, c2, c3};
}

// uniform in [0,1) with 24 random bits
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// stream ids keep the different random draws of one step independent
enum RngStream : uint32_t { RNG_DROPOUT = 1, RNG_LABEL_GT = 2, RNG_LABEL_NOGT = 3 };

__device__ __forceinline__ float rng_uniform(uint64_t seed, uint32_t step, uint32_t stream,
                                             uint32_t index) {
  u32x4 r = philox(index, step, stream, 0x5043u, (uint32_t)seed, (uint32_t)(seed >> 32));
  return u01(r.x);
}


// ---------------------------------------------------------------------------
// f32 MFMA helpers shared by the point-MLP kernels
// ---------------------------------------------------------------------------
// LDS row strides (floats): K + 4 keeps the ds_read_b128 fragment reads of 32
// consecutive rows conflict-free (row stride = 4 banks mod 64).
constexpr int S64 = 68;
constexpr int S128 = 132;

// One 32x32 f32 MFMA tile over K (multiple of 8) with the k-permuted fragment
// scheme: for k-group g, lane half h supplies k = 8g + 4h + j at MFMA step j, so
// each lane reads one float4 of A (LDS) and one float4 of B per 4 MFMAs.
template <int K>
__device__ __forceinline__ f32x16 mfma_rows_x_wt(const float* __restrict__ a_lds, int a_stride,
                                                 const f32x4* bfrag, f32x16 acc, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int g = 0; g < K / 8; ++g) {
    f32x4 a = *reinterpret_cast<const f32x4*>(a_lds + r * a_stride + 8 * g + 4 * h);
    acc = mfma32(a.x, bfrag[g].x, acc);
    acc = mfma32(a.y, bfrag[g].y, acc);
    acc = mfma32(a.z, bfrag[g].z, acc);
    acc = mfma32(a.w, bfrag[g].w, acc);
  }
  return acc;
}

// B fragments for output channels [o0, o0+32) of a row-major weight W[O][K].
template <int K>
__device__ __forceinline__ void load_bfrag(const float* __restrict__ w, int o0, int lane,
                                           f32x4* bfrag) {
  const int r = lane & 31, h = lane >> 5;
  const float* row = w + (size_t)(o0 + r) * K + 4 * h;
#pragma unroll
  for (int g = 0; g < K / 8; ++g) bfrag[g] = *reinterpret_cast<const f32x4*>(row + 8 * g);
}

// NaN-propagating "v beats best" (torch.max returns a NaN if one is present;
// ties keep the earlier index because points arrive in increasing order).
__device__ __forceinline__ bool beats(float v, float best) {
  return v > best || (v != v && best == best);
}

// conv1 (3 -> 64) + ReLU of one point, in the fixed fma order shared by the
// forward and the backward recompute (bit-identical results).
__device__ __forceinline__ float conv1_point(float wa, float wb, float wc, float bb, float p0,
                                             float p1, float p2) {
  const float v = fmaf(wc, p2, fmaf(wb, p1, fmaf(wa, p0, bb)));
  return v > 0.f ? v : 0.f;
}

// Work added to a linear-backward launch (linear.hip): an extra weight-gradient
// job dw[N][K] (+ db) = sum over the first m_w rows of dy^T x (no activation,
// no dropout), and a fixed-order sum of red_cnt slabs of red_n floats.
// torch.optim.Adam, single-tensor path (train_classification.py:110-122):
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2)
//   p.addcdiv_(m, sqrt(v)/sqrt(1-b2^t) + eps, value=-lr/(1-b1^t))
struct AdamHp {
  float w1, b2, w2, bc2s, eps, step;
};
__device__ __forceinline__ AdamHp adam_hp(const int32_t* step_count, int step_offset, float b1,
                                          float b2, float eps, float lr) {
  const double t = (double)(*step_count + step_offset);
  const float bc1 = (float)(1.0 - pow((double)b1, t));
  AdamHp h;
  h.bc2s = (float)sqrt(1.0 - pow((double)b2, t));
  h.step = (float)((double)lr / (double)bc1);
  h.w1 = 1.f - b1;
  h.w2 = 1.f - b2;
  h.b2 = b2;
  h.eps = eps;
  return h;
}
// Every rounding is explicit (no contraction left to the compiler), so the Adam
// fused into k_feat_bwd_finish and the standalone k_adam of the data-parallel
// path give bitwise the same parameters whatever code surrounds them.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHp& h) {
  m = __fmaf_rn(h.w1, __fsub_rn(g, m), m);
  v = __fmaf_rn(v, h.b2, __fmul_rn(h.w2, __fmul_rn(g, g)));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), h.bc2s), h.eps);
  p = __fmaf_rn(-h.step, __fdiv_rn(m, denom), p);
}

// Adam riding along the feature backward: the generator's conv1..conv4
// parameters in k_feat_bwd_finish as their gradients are formed, the
// parameters whose gradients are already final (G from fc1 on, all of D) in
// trailing workgroups of k_feat_bwd_chunk.
struct FinAdam {
  int on;
  float* gp; float* gm; float* gv; const float* gg;  // generator flat buffers
  int64_t g_rest0, g_n;                             // G [g_rest0, g_n) in the extra workgroups
  float* dp; float* dm; float* dv; const float* dg;  // discriminator (d_n = 0: none)
  int64_t d_n;
  float lr_g, lr_d, b1, b2, eps;
  const int32_t* step_count;
  int step_offset;
};

// The device jitter of a gathered batch point (dataset/modelNetData.py:80-91,
// jitter_point_cloud: clip(sigma * randn, -clip, clip) per coordinate): the
// point's row tg in the global batch keys a Philox draw whose two uniform
// pairs give, by Box-Muller, the normals of coordinates 0, 1, 2.  Coordinate d
// alone costs the same operations as all three do for it, so a thread per
// coordinate (k_point_mlp's folded gather) and a thread per point
// (k_gather_clouds) produce the same bits.
constexpr uint32_t RNG_JITTER = 4;
__device__ __forceinline__ float jitter_normal(uint64_t seed, uint32_t step, int64_t tg, int d) {
  const u32x4 r = philox((uint32_t)tg, step, RNG_JITTER, (uint32_t)(tg >> 32), (uint32_t)seed,
                         (uint32_t)(seed >> 32));
  // Box-Muller on two uniform pairs -> 4 normals (3 used)
  if (d < 2) {
    const float u1 = fmaxf(u01(r.x), 1e-7f), u2 = u01(r.y);
    const float m1 = sqrtf(-2.f * logf(u1)), a1 = 6.28318530718f * u2;
    return d == 0 ? m1 * cosf(a1) : m1 * sinf(a1);
  }
  const float u3 = fmaxf(u01(r.z), 1e-7f), u4 = u01(r.w);
  const float m2 = sqrtf(-2.f * logf(u3)), a2 = 6.28318530718f * u4;
  return m2 * cosf(a2);
}
__device__ __forceinline__ float jitter_coord(float x, float sigma, float clip, float z) {
  return x + fminf(fmaxf(sigma * z, -clip), clip);
}

// A step's input batches gathered by its first launch (pcadv_adv_args.gather):
// job 0 the clouds [0, split) of the feature forward, job 1 the rest.
struct GatherFold {
  pcadv_gather_job j[2];
  int n;
};

// The end of a graph-replayed training iteration (pcadv_iter_epilogue, or
// folded into the step's last launch through pcadv_adv_args.epi_*): every
// counter += 1 (the loaders' RNG steps and batch cursors) and, with a ring,
// losses[0..nl) into slot (*ring_count % slots), *ring_count += 1.  Called by
// the threads 0..63 of a workgroup: the count is read once and broadcast from
// the first lane (readfirstlane), and lane 0 stores the increment after that
// read, so the slot every writing lane (lane < nl <= 32) uses is the value
// before the increment also where a workgroup's first 64 threads were split
// over two wavefronts.
struct IterEpi {
  int32_t* counters;
  int ncounters;
  const float* losses;
  int nl;
  float* ring;
  int slots;
  int32_t* ring_count;
};
__device__ __forceinline__ void iter_epi_wave(const IterEpi& e, int lane) {
  if (e.ring && e.ring_count) {
    const int32_t cnt = __builtin_amdgcn_readfirstlane(*e.ring_count);
    const int slot = (int)((uint32_t)cnt % (uint32_t)e.slots);
    if (lane < e.nl) e.ring[(size_t)slot * e.nl + lane] = e.losses[lane];
    if (lane == 0) *e.ring_count = cnt + 1;
  }
  if (lane < e.ncounters) e.counters[lane] += 1;
}

// extra weight-gradient job: dw[N][K] (+ db) = sum over rows m < m_w of
// dz[m][N]^T x[m][K] (dz stored as is: no activation, no dropout)
struct LinBwdJob {
  const float* dz;
  const float* x;
  float* dw;
  float* db;
  int m_w, N, K;
};
constexpr int LB_MAXJOBS = 3;
struct LinBwdExtra {
  LinBwdJob job[LB_MAXJOBS];
  int njobs;
  const float* red_src;
  float* red_dst;
  int red_n, red_cnt;
  int red_ld;  // floats between slabs (0: red_n)
  // data-gradient output mask: dx *= act'(x) (* dx_mask * dx_keep), dx then
  // being the layer below's dz (its backward runs with act NONE, no dropout)
  int dx_act;
  const float* dx_mask;
  float dx_keep;
  // chained product of the data gradient's rows >= chain_row0 with the next
  // layer down's weight W' [K][chain_n] (row-major): per 16-column tile ct of
  // dx, chain_out[ct][m - chain_row0][j] = sum_{c in tile} dx[m][c] W'[c][j].
  // The consumer sums the K / 16 tile partials (the discriminator conv1 input
  // gradient of the adversarial rows, k_head_bwd).
  const float* chain_w;
  float* chain_out;
  int chain_row0, chain_n;
  // Adam over parameters whose gradients are final before this launch, in
  // trailing blocks (adam.on): the generator's [g_rest0, g_n) and the
  // discriminator's [0, d_n) of adam's flat buffers
  FinAdam adam;
};
int launch_linear_bwd(const float* dy, const float* y, int act, const float* mask,
                      const int32_t* step, uint64_t seed, float p, const float* x, const float* w,
                      float* dx, float* dw, float* db, int M, int m_w, int N, int K,
                      hipStream_t s, const LinBwdExtra* extra = nullptr);

}  // namespace pcadv

#define PC_HIP_CHECK_LAUNCH(what)                                              \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess) {                                                    \
      pcadv::set_error("%s: %s", what, hipGetErrorString(e_));                 \
      return PCADV_EHIP;                                                       \
    }                                                                          \
  } while (0)

#define PC_REQUIRE(cond, ...)                                                  \
  do {                                                                         \
    if (!(cond)) {                                                             \
      pcadv::set_error(__VA_ARGS__);                                           \
      return PCADV_EINVAL;                                                     \
    }                                                                          \
  } while (0)

// Dense point-wise GEMM engine for the segmentation net (models/pointnet.py:
// 261-317: conv1..conv6 and fc1..fc4 are per-point linear maps over B*N rows)
// on gfx950.
//
//   C[m][n] = sum_k A[m][k] B[n][k]      (+ bias, ReLU, accumulate, or a
//                                          max-over-points screening epilogue)
//
// f32 operands are split into bf16 planes while they are staged into LDS and
// multiplied as bf16 MFMA products with f32 accumulation: three products of
// hi/lo splits (relative error <= ~1.2e-5 of sum|a b|, 1/3 of the bf16 matrix
// rate = 5.3x the f32 MFMA rate) for the forward, six of hi/mid/lo splits
// (f32-level accuracy, 2.7x the f32 MFMA rate) for the gradients, whose sums
// over 10^4-10^5 points cancel heavily.
//
// Layouts (template TA / TB): A[m][k] at a[m*lda + k] (TA = 0) or a[k*lda + m]
// (TA = 1, i.e. A^T stored); B[n][k] at b[n*ldb + k] (TB = 0: a weight [out][in])
// or b[k*ldb + n] (TB = 1).  Forward: TA = 0, TB = 0.  Data gradient dX = dZ W:
// TA = 0, TB = 1.  Weight gradient dW = dZ^T X: TA = 1, TB = 1, split over the
// point axis into fixed-order slabs (k_slab_sum).
//
// An optional output mask zeroes C where a mask matrix Y (stored like C) is
// not > 0: relu'(Y) applied by the producer of dZ = dY relu'(Y), so that every
// consumer (the weight gradient, the next data gradient, the bias sums) reads
// dZ already masked.
#include "common.h"
#include <type_traits>

namespace pcadv {

#define PC_TRY_GEMM(call)        \
  do {                           \
    int rc_ = (call);            \
    if (rc_ != PCADV_OK) return rc_; \
  } while (0)

constexpr int GM_BM = 128, GM_BN = 128, GM_BK = 32;
constexpr int GM_T = 256;   // 4 waves, 2 x 2, each 64 x 64 of C
constexpr int GM_S = 40;    // bf16 row stride of the staged tiles (80 B: conflict-free b128 reads)

typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4g __attribute__((ext_vector_type(4)));

struct GemmLds {
  alignas(16) __bf16 a[3][GM_BM * GM_S];  // [hi, (mid,) lo][m][k]
  alignas(16) __bf16 b[3][GM_BN * GM_S];  // [hi, (mid,) lo][n][k]
};

// f32 -> NPL bf16 planes summing to it (round-to-nearest splits): NPL = 2
// (hi, lo: 16 significant bits) or 3 (hi, mid, lo: the whole f32 significand)
template <int NPL>
__device__ __forceinline__ void split_planes(float v, __bf16 (&o)[3]) {
  o[0] = (__bf16)v;
  const float r1 = v - (float)o[0];
  o[1] = (__bf16)r1;
  if (NPL == 3) o[2] = (__bf16)(r1 - (float)o[1]);
}

struct GemmP {
  const float* a; long long lda;
  const float* b; long long ldb;
  float* c; long long ldc;
  const float* cmask; long long ldm;  // nullable: C *= [cmask > 0], stored like C (stride ldm)
  const float* bias;               // [N] or null
  const float* bias_rows;          // [M / rows_per_group][N] or null
  int rows_per_group;               // bias_rows groups; mode 2: points per cloud
  int M, N, K;
  int relu, accumulate;
  int avec, bvec;                  // 16-B vector loads allowed (aligned base, ld % 4 == 0)
  int cvec;                        // the epilogue's C / bias / bias_rows / mask allow 16-B access
  // k range of slab z (grid.z): group z / zpg of grp rows, piece z % zpg of
  // ksplit_len rows (weight gradients: the point axis in fixed-order slabs)
  int grp, zpg, ksplit_len;
  long long slab_stride;           // floats between slabs
  float* csum;                     // TA = 1: per-slab column sums of A ([z][M]) or null
  // TA / TB = 2: the operand given as its bf16 hi / lo planes ([m][k] / [n][k],
  // row stride in elements), split once by its producer: staged as plain
  // copies (no VALU split per tile)
  const __bf16* ap[2]; long long ldap;
  const __bf16* bp[3]; long long ldbp;  // TB = 3: hi, mid, lo (the three-way split)
  __bf16* cp[2]; long long ldcp;    // nullable: the epilogue also writes C's hi / lo planes
  // max-over-points screening epilogue (mode 2): per (row tile, column) top-2
  int2* part;                      // [M / BM][N] screening keys
};

__device__ __forceinline__ f32x16 mfma_bf16g(bf16x8g a, bf16x8g b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// screening keys (as k_conv4_max, feat_fused.hip): the f32 value as an
// order-preserving int32 with 127 - (row within the 128-row tile) in the low
// 7 bits, so v_max_i32 / v_med3_i32 keep the top-2 (value, row), lower row
// first on equal truncated values
__device__ __forceinline__ int gkey(float v, int row) {
  const int b = __float_as_int(v);
  const int ord = b ^ ((b >> 31) & 0x7fffffff);
  return (ord & ~127) | (127 - row);
}
constexpr int GKEY_NONE = (int)0x80000000;

// NP = 3: three products of hi/lo splits (relative error <= ~1.2e-5 of
// sum|a b|); NP = 6: six products of hi/mid/lo splits (h h, h m, m h, h l, m m,
// l h), f32-level accuracy (the gradients, whose sums cancel heavily).
//
// Main loop: the f32 tiles are staged through registers two tiles ahead (two
// register sets), so two 32 KB tiles per workgroup are in flight while the
// MFMAs of the current one run; each tile is split into its bf16 planes once,
// on the way into LDS.  Transposed operands (TA / TB = 1: the reduction axis is
// the slow one) are read as 4 (k) x 4 (m) blocks per thread and written as
// 4-k runs (ds_write_b64) of each plane.
// The same rows without a mask or an accumulate target (the forward layers:
// bias, per-group bias, ReLU, planes): loads at their use, which measured
// faster there than the batched form below.
template <int MODE>
__device__ __forceinline__ void epilogue_rows_plain(const GemmP& p, float* C, const float* stage,
                                                    int es, int c4, int row0, int rstep, int nit,
                                                    int m0, int n) {
#pragma unroll 2
  for (int it = 0; it < nit; ++it) {
    const int row = row0 + rstep * it;
    const int m = m0 + row;
    if (m >= p.M) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(&stage[row * es + c4]);
    float* dst = C + (size_t)m * p.ldc + n;
    const float* br = p.bias_rows ? p.bias_rows + (size_t)(m / p.rows_per_group) * p.N + n : nullptr;
    if (p.cvec && n + 3 < p.N) {
      if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + n);
      if (br) v += *reinterpret_cast<const f32x4*>(br);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (p.relu) v[t] = v[t] > 0.f ? v[t] : 0.f;
      *reinterpret_cast<f32x4*>(dst) = v;
      if (p.cp[0]) {  // the hi / lo planes the next layer stages (ldcp % 4 == 0)
        bf16x4g hv, lv;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          hv[t] = (__bf16)v[t];
          lv[t] = (__bf16)(v[t] - (float)hv[t]);
        }
        const size_t pofs = (size_t)m * p.ldcp + n;
        *reinterpret_cast<bf16x4g*>(p.cp[0] + pofs) = hv;
        *reinterpret_cast<bf16x4g*>(p.cp[1] + pofs) = lv;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (n + t >= p.N) break;
        float x = v[t];
        if (p.bias) x += p.bias[n + t];
        if (br) x += br[t];
        if (p.relu) x = x > 0.f ? x : 0.f;
        dst[t] = x;
        if (p.cp[0]) {
          const __bf16 hx = (__bf16)x;
          p.cp[0][(size_t)m * p.ldcp + n + t] = hx;
          p.cp[1][(size_t)m * p.ldcp + n + t] = (__bf16)(x - (float)hx);
        }
      }
    }
  }
}

// Epilogue rows of a staged half tile: this thread's 4 columns n.. of rows
// row0 + rstep * it (it < NIT), C (+)= staged + bias + per-group bias, ReLU,
// output mask, optional bf16 hi / lo planes.  Every load of the NIT rows (the
// per-group bias, the accumulate target, the mask) is a buffer load issued
// before the first use (masked rows read zeros past the buffer's end); the
// per-row `if (present) load` form drained each load before the next (three
// L2 / HBM round trips per row: the masked data gradients and the accumulating
// GEMMs use this form).  Same additions in the same order as before.
template <int MODE, int NIT>
__device__ __forceinline__ void epilogue_rows(const GemmP& p, float* C, const float* stage, int es,
                                              int c4, int row0, int rstep, int m0, int n) {
  constexpr uint32_t OOB = 0x80000000u;
  auto opq = [](uint32_t o) {
    asm("" : "+v"(o));
    return o;
  };
  auto ld4 = [](__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  };
  auto rs = [](const void* b) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(b), (short)0, 0x7fffffff, 0x00020000);
  };
  const bool nv = p.cvec && n + 3 < p.N;  // this thread's columns as one 16-B vector
  // (each operand's loads under one launch-uniform branch: none are issued
  // for an absent operand)
  f32x4 bv = {0.f, 0.f, 0.f, 0.f};
  if (p.bias) bv = ld4(rs(p.bias), opq(nv ? (uint32_t)n * 4u : OOB));
  f32x4 brv[NIT], dv[NIT], mv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) brv[it] = dv[it] = mv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (p.bias_rows) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int m = m0 + row0 + rstep * it;
      brv[it] = ld4(rs(p.bias_rows),
                    opq(nv && m < p.M ? (uint32_t)((m / p.rows_per_group) * p.N + n) * 4u : OOB));
    }
  }
  if (MODE == 1) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int m = m0 + row0 + rstep * it;
      dv[it] = ld4(rs(C), opq(nv && m < p.M ? (uint32_t)((long long)m * p.ldc + n) * 4u : OOB));
    }
  }
  if (p.cmask) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int m = m0 + row0 + rstep * it;
      mv[it] = ld4(rs(p.cmask), opq(nv && m < p.M ? (uint32_t)((long long)m * p.ldm + n) * 4u : OOB));
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int row = row0 + rstep * it;
    const int m = m0 + row;
    if (m >= p.M) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(&stage[row * es + c4]);
    float* dst = C + (size_t)m * p.ldc + n;
    if (nv) {
      if (p.bias) v += bv;
      if (p.bias_rows) v += brv[it];
      if (MODE == 1) v += dv[it];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (p.relu) v[t] = v[t] > 0.f ? v[t] : 0.f;
        if (p.cmask && !(mv[it][t] > 0.f)) v[t] = 0.f;
      }
      *reinterpret_cast<f32x4*>(dst) = v;
      if (p.cp[0]) {  // the hi / lo planes the next layer stages (ldcp % 4 == 0)
        bf16x4g hv, lv;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          hv[t] = (__bf16)v[t];
          lv[t] = (__bf16)(v[t] - (float)hv[t]);
        }
        const size_t pofs = (size_t)m * p.ldcp + n;
        *reinterpret_cast<bf16x4g*>(p.cp[0] + pofs) = hv;
        *reinterpret_cast<bf16x4g*>(p.cp[1] + pofs) = lv;
      }
    } else {  // ragged right edge or unaligned output: element by element
      const float* br = p.bias_rows ? p.bias_rows + (size_t)(m / p.rows_per_group) * p.N + n : nullptr;
      const float* mk = p.cmask ? p.cmask + (size_t)m * p.ldm + n : nullptr;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (n + t >= p.N) break;
        float x = v[t];
        if (p.bias) x += p.bias[n + t];
        if (br) x += br[t];
        if (MODE == 1) x += dst[t];
        if (p.relu) x = x > 0.f ? x : 0.f;
        if (mk && !(mk[t] > 0.f)) x = 0.f;
        dst[t] = x;
        if (p.cp[0]) {
          const __bf16 hx = (__bf16)x;
          p.cp[0][(size_t)m * p.ldcp + n + t] = hx;
          p.cp[1][(size_t)m * p.ldcp + n + t] = (__bf16)(x - (float)hx);
        }
      }
    }
  }
}

// VEC bit 0 / bit 1: A / B staged by 16-byte loads (vector-aligned, no
// vector straddles an edge), else by dword loads
// The body of one workgroup of k_gemm_x3: linear block id lin of a
// gx x gy x gz grid (k_gemm_x3 passes its own; the pair kernel below runs two
// GEMMs' workgroups in one launch)
template <int TA, int TB, int MODE, int NP, int VEC>
__device__ __forceinline__ void gemm_x3_body(const GemmP& p, int lin, int gx, int gy, int gzn) {
  constexpr int NPL = NP == 6 ? 3 : 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GemmLds& L = *reinterpret_cast<GemmLds*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: the workgroups one XCD runs (linear id = xcd mod 8)
  // take consecutive tiles with the column tile fastest, so the column tiles
  // sharing a row tile of A run together on one XCD and read it from its L2
  int tx, ty, tz;
  {
    const int n = gx * gy * gzn;
    const int xcd = lin & 7, q = n >> 3, rr = n & 7;
    const int t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (lin >> 3);
    tz = t / (gx * gy);
    const int rem = t % (gx * gy);
    // wide outputs (>= 16 column tiles: conv6's 2048) go column-group-major in
    // groups of 8, so the B tiles a group shares stay in L2 while A streams by
    // (all 16 at once plus the A tiles in flight overflow one XCD's 4 MB)
    constexpr int CG = 8;
    if (gy >= 2 * CG && gy % CG == 0) {
      const int g = rem / (gx * CG), w = rem % (gx * CG);
      tx = w / CG;
      ty = g * CG + w % CG;
    } else {
      tx = rem / gy;
      ty = rem % gy;
    }
  }
  const int n0 = ty * GM_BN;
  // mode 2: tx = (cloud, row tile of that cloud); rows never straddle clouds
  const int T2 = MODE == 2 ? (p.rows_per_group + GM_BM - 1) / GM_BM : 1;
  const int cl = MODE == 2 ? tx / T2 : 0;
  const int m0 = MODE == 2 ? (tx % T2) * GM_BM : tx * GM_BM;
  const int Mlim = MODE == 2 ? p.rows_per_group : p.M;
  const float* Ab = MODE == 2 && TA != 2 ? p.a + (size_t)cl * p.rows_per_group * p.lda : p.a;
  const size_t aoff2 = MODE == 2 ? (size_t)cl * p.rows_per_group * p.ldap : 0;
  const int gz = tz / p.zpg, sz = tz % p.zpg;
  const int kz0 = gz * p.grp + sz * p.ksplit_len;
  const int kz1 = min(min(p.K, (gz + 1) * p.grp), kz0 + p.ksplit_len);
  float* C = p.c + (size_t)tz * p.slab_stride;
  const bool do_csum = TA == 1 && p.csum != nullptr && ty == 0;

  // one operand tile (128 x 32 f32 = 4096 values, 16 per thread)
  //   [m][k] layout: thread = (row tid >> 1, 16 k at 16 (tid & 1))
  //   [k][m] layout: thread = (4 k at 4 (tid & 7), 4 m at 4 (tid >> 3))
  // Buffer loads with no data-dependent selects or branches: a masked vector
  // or element gets an offset past the buffer's end and reads zeros (the old
  // `if (in range) load` form made the compiler wait out each load before the
  // next one).  Vector loads only where no vector straddles the edge (vec and
  // the edge a multiple of 4, a launch constant), else four dword loads.
  constexpr uint32_t OOB = 0x80000000u;
  // an opaque copy of a masked offset: the compiler otherwise turns the mask
  // into branches around duplicated loads (divergent control flow that drains
  // the loads in flight)
  auto opq = [](uint32_t o) {
    asm("" : "+v"(o));
    return o;
  };
  auto rsrc = [](const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
  };
  // (planes: hi and lo resources, A's at this cloud's rows in mode 2)
  const __amdgpu_buffer_rsrc_t ars = rsrc(TA == 2 ? (const void*)(p.ap[0] + aoff2) : (const void*)Ab);
  const __amdgpu_buffer_rsrc_t arsl = rsrc(TA == 2 ? (const void*)(p.ap[1] + aoff2) : (const void*)Ab);
  const __amdgpu_buffer_rsrc_t brs = rsrc(TB >= 2 ? (const void*)p.bp[0] : (const void*)p.b);
  const __amdgpu_buffer_rsrc_t brsl = rsrc(TB >= 2 ? (const void*)p.bp[1] : (const void*)p.b);
  // TB = 3: B as the hi / mid / lo planes of its three-way split (split once per
  // step by pcadv_split_bf3, bitwise split_planes<3> of the f32 value), staged
  // as plain copies; same LDS image, so the same MFMAs on the same values
  const __amdgpu_buffer_rsrc_t brs3 = rsrc(TB == 3 ? (const void*)p.bp[2] : (const void*)p.b);
  constexpr bool vecA = (VEC & 1) != 0, vecB = (VEC & 2) != 0;
  auto load_rows = [&](f32x4 (&v)[4], const __amdgpu_buffer_rsrc_t& rs, long long ld, int row0,
                       int rlim, int k0, auto VECT) {
    constexpr bool vec = decltype(VECT)::value;
    const int row = row0 + (tid >> 1), kk = k0 + 16 * (tid & 1);
    const bool rok = row < rlim;
    const uint32_t rb = rok ? (uint32_t)((long long)row * ld) : 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kk + 4 * j;
      if constexpr (vec) {
        const uint32_t off = opq(rok && k >= kz0 && k < kz1 ? (rb + (uint32_t)k) * 4u : OOB);
        v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int kt = k + t;
          const uint32_t off = opq(rok && kt >= kz0 && kt < kz1 ? (rb + (uint32_t)kt) * 4u : OOB);
          v[j][t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        }
      }
    }
  };
  auto load_cols = [&](f32x4 (&v)[4], const __amdgpu_buffer_rsrc_t& rs, long long ld, int col0,
                       int clim, int k0, auto VECT) {
    constexpr bool vec = decltype(VECT)::value;
    const int col = col0 + 4 * (tid >> 3), kk = k0 + 4 * (tid & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kk + j;
      const bool kok = k >= kz0 && k < kz1;
      const uint32_t kb = kok ? (uint32_t)((long long)k * ld) : 0u;
      if constexpr (vec) {
        const uint32_t off = opq(kok && col < clim ? (kb + (uint32_t)col) * 4u : OOB);
        v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t off = opq(kok && col + t < clim ? (kb + (uint32_t)(col + t)) * 4u : OOB);
          v[j][t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        }
      }
    }
  };
  auto store_rows = [&](const f32x4 (&v)[4], __bf16 (*planes)[GM_BM * GM_S]) {
    const int row = tid >> 1, kk = 16 * (tid & 1);
    bf16x8g pv[3][2];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      __bf16 o[3];
      split_planes<NPL>(v[j >> 2][j & 3], o);
#pragma unroll
      for (int q = 0; q < NPL; ++q) pv[q][j >> 3][j & 7] = o[q];
    }
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      *reinterpret_cast<bf16x8g*>(&planes[q][row * GM_S + kk]) = pv[q][0];
      *reinterpret_cast<bf16x8g*>(&planes[q][row * GM_S + kk + 8]) = pv[q][1];
    }
  };
  auto store_cols = [&](const f32x4 (&v)[4], __bf16 (*planes)[GM_BM * GM_S]) {
    const int col = 4 * (tid >> 3), kk = 4 * (tid & 7);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x4g pv[3];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __bf16 o[3];
        split_planes<NPL>(v[j][i], o);
#pragma unroll
        for (int q = 0; q < NPL; ++q) pv[q][j] = o[q];
      }
#pragma unroll
      for (int q = 0; q < NPL; ++q)
        *reinterpret_cast<bf16x4g*>(&planes[q][(col + i) * GM_S + kk]) = pv[q];
    }
  };
  // planes: thread = (row tid >> 1, 16 k at 16 (tid & 1)); v[0..1] = hi, v[2..3]
  // = lo, each 8 bf16 carried as 16 raw bytes (K % 16 == 0, ld % 8 == 0)
  auto load_planes = [&](f32x4 (&v)[4], const __amdgpu_buffer_rsrc_t& rh,
                         const __amdgpu_buffer_rsrc_t& rl, long long ld, int row0, int rlim, int k0) {
    const int row = row0 + (tid >> 1), k = k0 + 16 * (tid & 1);
    const bool ok = row < rlim && k >= kz0 && k < kz1;
    const uint32_t o = opq(ok ? (uint32_t)((long long)row * ld + k) * 2u : OOB);
    v[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, o, 0, 0));
    v[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, o + 16u, 0, 0));
    v[2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, o, 0, 0));
    v[3] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, o + 16u, 0, 0));
  };
  // three planes: v[0..1] = hi, v[2..3] = mid, v[4..5] = lo
  auto load_planes3 = [&](f32x4 (&v)[6], long long ld, int row0, int rlim, int k0) {
    const int row = row0 + (tid >> 1), k = k0 + 16 * (tid & 1);
    const bool ok = row < rlim && k >= kz0 && k < kz1;
    const uint32_t o = opq(ok ? (uint32_t)((long long)row * ld + k) * 2u : OOB);
    v[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(brs, o, 0, 0));
    v[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(brs, o + 16u, 0, 0));
    v[2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(brsl, o, 0, 0));
    v[3] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(brsl, o + 16u, 0, 0));
    v[4] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(brs3, o, 0, 0));
    v[5] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(brs3, o + 16u, 0, 0));
  };
  auto store_planes3 = [&](const f32x4 (&v)[6], __bf16 (*planes)[GM_BM * GM_S]) {
    const int row = tid >> 1, kk = 16 * (tid & 1);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      *reinterpret_cast<f32x4*>(&planes[q][row * GM_S + kk]) = v[2 * q];
      *reinterpret_cast<f32x4*>(&planes[q][row * GM_S + kk + 8]) = v[2 * q + 1];
    }
  };
  auto store_planes = [&](const f32x4 (&v)[4], __bf16 (*planes)[GM_BM * GM_S]) {
    const int row = tid >> 1, kk = 16 * (tid & 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *reinterpret_cast<f32x4*>(&planes[q][row * GM_S + kk]) = v[2 * q];
      *reinterpret_cast<f32x4*>(&planes[q][row * GM_S + kk + 8]) = v[2 * q + 1];
    }
  };
  float cs[4] = {0.f, 0.f, 0.f, 0.f};  // TA = 1: this thread's column sums of A
  auto load_tile = [&](f32x4 (&ra)[4], auto& rb, int k0) {
    if (TA == 2) load_planes(ra, ars, arsl, p.ldap, m0, Mlim, k0);
    else if (TA == 0) load_rows(ra, ars, p.lda, m0, Mlim, k0, std::integral_constant<bool, vecA>{});
    else load_cols(ra, ars, p.lda, m0, Mlim, k0, std::integral_constant<bool, vecA>{});
    if constexpr (TB == 3) load_planes3(rb, p.ldbp, n0, p.N, k0);
    else if constexpr (TB == 2) load_planes(rb, brs, brsl, p.ldbp, n0, p.N, k0);
    else if constexpr (TB == 0) load_rows(rb, brs, p.ldb, n0, p.N, k0, std::integral_constant<bool, vecB>{});
    else load_cols(rb, brs, p.ldb, n0, p.N, k0, std::integral_constant<bool, vecB>{});
  };
  auto store_tile = [&](const f32x4 (&ra)[4], const auto& rb) {
    if (TA == 2) store_planes(ra, L.a);
    else if (TA == 0) store_rows(ra, L.a);
    else {
      store_cols(ra, L.a);
      if (do_csum) {
#pragma unroll
        for (int i = 0; i < 4; ++i) cs[i] += ((ra[0][i] + ra[1][i]) + ra[2][i]) + ra[3][i];
      }
    }
    if constexpr (TB == 3) store_planes3(rb, L.b);
    else if constexpr (TB == 2) store_planes(rb, L.b);
    else if constexpr (TB == 0) store_rows(rb, L.b);
    else store_cols(rb, L.b);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  auto mfma_tile = [&]() {
#pragma unroll
    for (int kb = 0; kb < GM_BK / 16; ++kb) {
      bf16x8g fa[3][2], fb[3][2];  // [plane][tile]
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ar = (64 * wm + 32 * t + r) * GM_S + 16 * kb + 8 * h;
        const int br = (64 * wn + 32 * t + r) * GM_S + 16 * kb + 8 * h;
#pragma unroll
        for (int q = 0; q < NPL; ++q) {
          fa[q][t] = *reinterpret_cast<const bf16x8g*>(&L.a[q][ar]);
          fb[q][t] = *reinterpret_cast<const bf16x8g*>(&L.b[q][br]);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (NP == 6) {  // smallest terms first
            acc[i][j] = mfma_bf16g(fa[2][i], fb[0][j], acc[i][j]);
            acc[i][j] = mfma_bf16g(fa[1][i], fb[1][j], acc[i][j]);
            acc[i][j] = mfma_bf16g(fa[0][i], fb[2][j], acc[i][j]);
            acc[i][j] = mfma_bf16g(fa[1][i], fb[0][j], acc[i][j]);
            acc[i][j] = mfma_bf16g(fa[0][i], fb[1][j], acc[i][j]);
            acc[i][j] = mfma_bf16g(fa[0][i], fb[0][j], acc[i][j]);
          } else {
            acc[i][j] = mfma_bf16g(fa[1][i], fb[0][j], acc[i][j]);
            acc[i][j] = mfma_bf16g(fa[0][i], fb[1][j], acc[i][j]);
            acc[i][j] = mfma_bf16g(fa[0][i], fb[0][j], acc[i][j]);
          }
        }
    }
  };

  if constexpr ((VEC & 4) != 0) {
    // LDS-DMA form for plane operands (VEC bit 2; TA = TB = 2, whole tiles:
    // M, N % 128, K % 32, one k-range), as k_gemm_bf2_big<MODE, true>: two
    // 32 KB buffers of unpadded 64-B rows, the 16-B chunk XOR-swizzled by
    // (row >> 2) & 3 on the source address; wave w issues 8 of the tile's 32
    // buffer_load ... lds (operand i >> 2, plane (i >> 1) & 1, 16-row block
    // 2 w + (i & 1)); one barrier per tile between its two k-blocks
    static_assert(TA == 2 && TB == 2 && MODE != 2, "LDS-DMA staging: plane operands, modes 0 / 1");
    __bf16* const gl = reinterpret_cast<__bf16*>(smem);  // [buf][A hi, A lo, B hi, B lo][128 x 32]
    constexpr int PL = GM_BM * GM_BK;                     // bf16 per plane tile
    const int wsc = __builtin_amdgcn_readfirstlane(wave);
    const int lr = lane >> 2, lc = (lane & 3) ^ ((lane >> 4) & 3);
    const uint32_t alane = (uint32_t)(lr * p.ldap + 8 * lc) * 2u;
    const uint32_t blane = (uint32_t)(lr * p.ldbp + 8 * lc) * 2u;
    const uint32_t arow0 = (uint32_t)m0 * (uint32_t)p.ldap * 2u, brow0 = (uint32_t)n0 * (uint32_t)p.ldbp * 2u;
    auto issue = [&](int k0, int buf) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int opb = i >> 2, q = (i >> 1) & 1, rb16 = 2 * wsc + (i & 1);
        const __amdgpu_buffer_rsrc_t rs = opb ? (q ? brsl : brs) : (q ? arsl : ars);
        const uint32_t so = (opb ? brow0 + (uint32_t)(16 * rb16) * (uint32_t)p.ldbp * 2u
                                 : arow0 + (uint32_t)(16 * rb16) * (uint32_t)p.ldap * 2u) + (uint32_t)k0 * 2u;
        __bf16* dst = gl + (size_t)(buf * 4 + 2 * opb + q) * PL + 16 * rb16 * GM_BK;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16,
                                                 opb ? blane : alane, (int)so, 0, 0);
      }
    };
    // one k-block's fragments: [plane][tile] of A and B (32 VGPRs)
    auto read_kb = [&](int buf, int kb, bf16x8g (&fa)[2][2], bf16x8g (&fb)[2][2]) {
      const int c = 2 * kb + h;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ra_ = 64 * wm + 32 * t + r, rb_ = 64 * wn + 32 * t + r;
        const int oa = ra_ * GM_BK + 8 * (c ^ ((ra_ >> 2) & 3));
        const int ob = rb_ * GM_BK + 8 * (c ^ ((rb_ >> 2) & 3));
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          fa[q][t] = *reinterpret_cast<const bf16x8g*>(gl + (size_t)(buf * 4 + q) * PL + oa);
          fb[q][t] = *reinterpret_cast<const bf16x8g*>(gl + (size_t)(buf * 4 + 2 + q) * PL + ob);
        }
      }
    };
    auto mfma_kb = [&](const bf16x8g (&fa)[2][2], const bf16x8g (&fb)[2][2]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma_bf16g(fa[1][i], fb[0][j], acc[i][j]);
          acc[i][j] = mfma_bf16g(fa[0][i], fb[1][j], acc[i][j]);
          acc[i][j] = mfma_bf16g(fa[0][i], fb[0][j], acc[i][j]);
        }
    };
    const int nt = (kz1 - kz0) / GM_BK;
    bf16x8g fa0[2][2], fb0[2][2], fa1[2][2], fb1[2][2];
    issue(kz0, 0);
    __syncthreads();
    if (nt > 1) issue(kz0 + GM_BK, 1);
    read_kb(0, 0, fa0, fb0);
    read_kb(0, 1, fa1, fb1);
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      mfma_kb(fa0, fb0);
      if (t + 1 < nt) {
        __syncthreads();
        if (t + 2 < nt) issue(kz0 + (t + 2) * GM_BK, buf);
        read_kb(buf ^ 1, 0, fa0, fb0);
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_kb(fa1, fb1);
      if (t + 1 < nt) read_kb(buf ^ 1, 1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
  // one register set: tile t + 1 is loaded right after tile t is stored; the
  // sched_barrier keeps those loads ahead of tile t's MFMAs (as
  // k_gemm_bf2_big), so one tile's MFMAs cover the next tile's loads
  f32x4 ra[4], rb[TB == 3 ? 6 : 4];
  load_tile(ra, rb, kz0);
  for (int k0 = kz0; k0 < kz1; k0 += GM_BK) {
    __syncthreads();  // every wave is done reading the previous tile
    store_tile(ra, rb);
    __syncthreads();
    load_tile(ra, rb, k0 + GM_BK);
    __builtin_amdgcn_sched_barrier(0);
    mfma_tile();
  }
  }

  if (do_csum) {  // fixed-order reduction over the 8 k-lanes of each column group
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cs[i] += __shfl_xor(cs[i], 1);
      cs[i] += __shfl_xor(cs[i], 2);
      cs[i] += __shfl_xor(cs[i], 4);
    }
    const int col = m0 + 4 * (tid >> 3);
    if ((tid & 7) == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (col + i < Mlim) p.csum[(size_t)tz * p.M + col + i] = cs[i];
  }

  if constexpr (MODE == 2) {
    // screening epilogue: per column, the top-2 (value, row) of this tile's
    // 128 rows -> part[row tile][n]; the row's bias / ReLU are applied by the
    // exact re-evaluation (neither changes the order)
    __shared__ int2 red[2][GM_BN];  // the two wm halves of each column
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int k1 = GKEY_NONE, k2 = GKEY_NONE;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = 64 * wm + 32 * i + acc_row(e, lane);
          if (m0 + row < Mlim) {
            const int key = gkey(acc[i][j][e], row);
            k2 = max(min(key, k1), k2);
            k1 = max(k1, key);
          }
        }
      const int o1 = __shfl_xor(k1, 32), o2 = __shfl_xor(k2, 32);
      k2 = max(min(k1, o1), max(k2, o2));
      k1 = max(k1, o1);
      if (h == 0) red[wm][64 * wn + 32 * j + r] = make_int2(k1, k2);
    }
    __syncthreads();
    for (int c = tid; c < GM_BN; c += GM_T) {
      const int n = n0 + c;
      if (n >= p.N) continue;
      const int2 x = red[0][c], y = red[1][c];
      const int b2 = max(min(x.x, y.x), max(x.y, y.y));
      const int b1 = max(x.x, y.x);
      p.part[(size_t)tx * p.N + n] = make_int2(b1, b2);
    }
  } else {
    // epilogue through LDS, one 128 x 64 half of the tile at a time (each
    // wave's 32-column block j): rows are then written by 16 lanes x 4
    // consecutive columns, so C, the per-group bias and the mask move as
    // coalesced 16-B accesses with one address per row
    float* stage = reinterpret_cast<float*>(smem);
    constexpr int ES = 68;  // row stride (floats) of the staged half tile
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      __syncthreads();  // the MFMA operands / the previous half are no longer read
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          stage[(64 * wm + 32 * i + acc_row(e, lane)) * ES + 32 * wn + r] = acc[i][j][e];
      __syncthreads();
      const int c4 = 4 * (tid & 15);                 // staged column (0..60)
      const int n = n0 + 64 * (c4 >> 5) + 32 * j + (c4 & 31);
      if (MODE == 1 || p.cmask) epilogue_rows<MODE, 8>(p, C, stage, ES, c4, tid >> 4, 16, m0, n);
      else epilogue_rows_plain<MODE>(p, C, stage, ES, c4, tid >> 4, 16, 8, m0, n);
    }
  }
}

template <int TA, int TB, int MODE, int NP, int VEC>
__global__ void __launch_bounds__(GM_T)
k_gemm_x3(GemmP p) {
  gemm_x3_body<TA, TB, MODE, NP, VEC>(
      p, (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)), (int)gridDim.x,
      (int)gridDim.y, (int)gridDim.z);
}

// A weight gradient (six products, TA = TB = 1, slabs) and an independent data
// gradient (TA = 0, TB = 1, NPD = three or six products) in ONE launch: workgroups
// [0, n_first) run the first of the two, the rest the second (wfirst: the
// weight gradient first).  Each keeps its own grid geometry and XCD order, so
// every output is bitwise what its own launch gives; the pair saves a launch
// boundary and lets the two fill each other's idle CUs (the segmentation
// backward's per-layer weight and data gradients both read that layer's dz).
struct PairGeom { int n, gx, gy, gz; };
template <int VW, int MD, int VD, int NPD>
__global__ void __launch_bounds__(GM_T)
k_gemm_x3_pair(GemmP pw, PairGeom gw, GemmP pd, PairGeom gd, int wfirst) {
  const int b = (int)blockIdx.x;
  const int nfirst = wfirst ? gw.n : gd.n;
  const bool w = (b < nfirst) == (wfirst != 0);
  const int lin = b < nfirst ? b : b - nfirst;
  if (w) gemm_x3_body<1, 1, 0, 6, VW>(pw, lin, gw.gx, gw.gy, gw.gz);
  else gemm_x3_body<0, 1, MD, NPD, VD>(pd, lin, gd.gx, gd.gy, gd.gz);
}

// ---------------------------------------------------------------------------
// 256 x 256 tiles for the wide plane-operand GEMMs (conv5 -> 2048 with the
// max screening, conv4 -> 512): both operands given as bf16 hi / lo planes
// (TA = TB = 2), three products.  At 128 x 128 a workgroup streams 1 KB of
// planes per k for 16 K MACs; at 256 x 256 the same bytes feed 4x the MACs,
// which halves the L2 -> LDS bytes per FLOP (the 128-tile conv6 pulls ~2 GB
// per launch through L2).  Eight waves (2 x 4), each a 128 x 64 block of C
// as 4 x 2 accumulators of 32 x 32; one workgroup per CU.  Every output sums
// the same MFMAs in the same order as k_gemm_x3<2, 2, MODE, 3> (k-blocks in
// order, lo.hi + hi.lo + hi.hi), so the results are bitwise the same; the
// screening epilogue writes one top-2 record per 128-row half, the format
// k_max_combine reads from the 128-row kernel.
// ---------------------------------------------------------------------------
constexpr int GB_BM = 256, GB_BN = 256;
constexpr int GB_T = 512;
constexpr int GB_ES = 132;  // row stride (floats) of the staged 256 x 128 epilogue half
#ifndef PCADV_GEMM_BIG_DB
#define PCADV_GEMM_BIG_DB 1
#endif
constexpr int GB_NBUF = PCADV_GEMM_BIG_DB ? 2 : 1;  // LDS operand buffers (2: 160 KB, the whole LDS)
struct GemmBigLds {
  union {
    struct {
      alignas(16) __bf16 a[2][GB_BM * GM_S];  // [hi, lo][m][k]
      alignas(16) __bf16 b[2][GB_BN * GM_S];  // [hi, lo][n][k]
    } op[GB_NBUF];
    alignas(16) float stage[GB_BM * GB_ES];
  };
};

// LDS-DMA form (GL = true; whole tiles only: M % 256 == 0 per launch / cloud
// and K % 32 == 0): the planes go global -> LDS by buffer_load ... lds, no
// staging registers and no ds_write pass.  The image is lane-linear (one
// wave-instruction fills 1 KB = 16 rows of 64 B), so the fragment reads are
// kept conflict-free by an XOR swizzle of the 16-B chunk inside each row,
// chunk' = chunk ^ ((row >> 2) & 3), applied on the global source address.
struct GemmGlLds {
  union {
    struct {
      alignas(16) __bf16 a[2][GB_BM * GM_BK];  // [hi, lo][m][k], swizzled chunks
      alignas(16) __bf16 b[2][GB_BN * GM_BK];
    } op[2];
    alignas(16) float stage[GB_BM * GB_ES];
  };
};

template <int MODE, bool GL>
__global__ void __launch_bounds__(GB_T)
k_gemm_bf2_big(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GemmBigLds& L = *reinterpret_cast<GemmBigLds*>(smem);
  GemmGlLds& G = *reinterpret_cast<GemmGlLds*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 2, wn = wave & 3;
  // XCD-aware order (as k_gemm_x3): the workgroups of one XCD take consecutive
  // tiles, column tile fastest, so the column tiles of a row tile share its A
  int tx, ty;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const int n = gx * gy;
    const int lin = blockIdx.x + gx * blockIdx.y;
    const int xcd = lin & 7, q = n >> 3, rr = n & 7;
    const int t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (lin >> 3);
    tx = t / gy;
    ty = t % gy;
  }
  const int n0 = ty * GB_BN;
  // mode 2: tx = (cloud, 256-row tile of that cloud); rows never straddle clouds
  const int T2 = MODE == 2 ? p.rows_per_group / GB_BM : 1;
  const int cl = MODE == 2 ? tx / T2 : 0;
  const int m0 = MODE == 2 ? (tx % T2) * GB_BM : tx * GB_BM;
  const int Mlim = MODE == 2 ? p.rows_per_group : p.M;
  const size_t aoff = MODE == 2 ? (size_t)cl * p.rows_per_group * p.ldap : 0;
  const int K = p.K;

  // planes of one 256 x 32 tile: thread = (row tid >> 1, 16 k at 16 (tid & 1));
  // v[0..1] = hi, v[2..3] = lo, 8 bf16 each carried as 16 raw bytes.  Buffer
  // loads: a masked element (row past the matrix, k outside [0, K)) gets an
  // offset past the buffer's end and reads zeros, so no select waits on the
  // data (a select after the load made the compiler drain every load of the
  // prefetch right after issuing it); 32-bit offsets, no 64-bit addresses.
  const int lrow = tid >> 1, lk = 16 * (tid & 1);
  const __amdgpu_buffer_rsrc_t arsc[2] = {
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.ap[0] + aoff), (short)0, 0x7fffffff, 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.ap[1] + aoff), (short)0, 0x7fffffff, 0x00020000)};
  const __amdgpu_buffer_rsrc_t brsc[2] = {
      __builtin_amdgcn_make_buffer_rsrc((void*)p.bp[0], (short)0, 0x7fffffff, 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)p.bp[1], (short)0, 0x7fffffff, 0x00020000)};
  constexpr uint32_t OOB = 0x80000000u;  // >= num_records: the load returns zeros
  const bool arow_ok = m0 + lrow < Mlim, brow_ok = n0 + lrow < p.N;
  const uint32_t abase = (uint32_t)((m0 + lrow) * p.ldap + lk) * 2u;
  const uint32_t bbase = (uint32_t)((n0 + lrow) * p.ldbp + lk) * 2u;
  auto load_planes = [&](f32x4 (&v)[4], const __amdgpu_buffer_rsrc_t (&rs)[2], uint32_t base,
                         bool row_ok, int k0) {
    const int k = k0 + lk;
    const uint32_t off = row_ok && k >= 0 && k < K ? base + (uint32_t)k0 * 2u : OOB;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      v[2 * q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs[q], off, 0, 0));
      v[2 * q + 1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs[q], off + 16u, 0, 0));
    }
  };
  auto store_planes = [&](const f32x4 (&v)[4], __bf16 (*planes)[GB_BM * GM_S]) {
    const int row = tid >> 1, kk = 16 * (tid & 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *reinterpret_cast<f32x4*>(&planes[q][row * GM_S + kk]) = v[2 * q];
      *reinterpret_cast<f32x4*>(&planes[q][row * GM_S + kk + 8]) = v[2 * q + 1];
    }
  };
  auto load_tile = [&](f32x4 (&ra)[4], auto& rb, int k0) {
    load_planes(ra, arsc, abase, arow_ok, k0);
    load_planes(rb, brsc, bbase, brow_ok, k0);
  };
  auto store_tile = [&](const f32x4 (&ra)[4], const f32x4 (&rb)[4], int buf) {
    store_planes(ra, L.op[buf].a);
    store_planes(rb, L.op[buf].b);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  auto mfma_tile = [&](int buf) {
#pragma unroll
    for (int kb = 0; kb < GM_BK / 16; ++kb) {
      bf16x8g fb[2][2];  // [plane][j]
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int br = (64 * wn + 32 * j + r) * GM_S + 16 * kb + 8 * h;
#pragma unroll
        for (int q = 0; q < 2; ++q) fb[q][j] = *reinterpret_cast<const bf16x8g*>(&L.op[buf].b[q][br]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ar = (128 * wm + 32 * i + r) * GM_S + 16 * kb + 8 * h;
        const bf16x8g ah = *reinterpret_cast<const bf16x8g*>(&L.op[buf].a[0][ar]);
        const bf16x8g al = *reinterpret_cast<const bf16x8g*>(&L.op[buf].a[1][ar]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma_bf16g(al, fb[0][j], acc[i][j]);
          acc[i][j] = mfma_bf16g(ah, fb[1][j], acc[i][j]);
          acc[i][j] = mfma_bf16g(ah, fb[0][j], acc[i][j]);
        }
      }
    }
  };

  if constexpr (GL) {
    // wave w issues eight of the tile's 64 LDS-DMA loads, i < 8: operand
    // i >> 2 (A, B), plane (i >> 1) & 1, 16-row block 2 w + (i & 1) (operand
    // and plane compile-time, so the resources stay in SGPRs); lane l fills
    // row 16 block + l / 4, physical chunk l & 3 = logical chunk
    // (l & 3) ^ ((l >> 4) & 3) (the row's (row >> 2) & 3)
    const int lr = lane >> 2, lc = (lane & 3) ^ ((lane >> 4) & 3);
    const int wsc = __builtin_amdgcn_readfirstlane(wave);  // scalar: soffset and the LDS base (M0)
    const uint32_t alane = (uint32_t)(lr * p.ldap + 8 * lc) * 2u;
    const uint32_t blane = (uint32_t)(lr * p.ldbp + 8 * lc) * 2u;
    const uint32_t arow0 = (uint32_t)m0 * (uint32_t)p.ldap * 2u, brow0 = (uint32_t)n0 * (uint32_t)p.ldbp * 2u;
    auto issue = [&](int k0, int buf) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int opb = i >> 2, q = (i >> 1) & 1, rb16 = 2 * wsc + (i & 1);
        const __amdgpu_buffer_rsrc_t rs = opb ? brsc[q] : arsc[q];
        const uint32_t so = (opb ? brow0 + (uint32_t)(16 * rb16) * (uint32_t)p.ldbp * 2u
                                 : arow0 + (uint32_t)(16 * rb16) * (uint32_t)p.ldap * 2u) + (uint32_t)k0 * 2u;
        __bf16* dst = (opb ? G.op[buf].b[q] : G.op[buf].a[q]) + 16 * rb16 * GM_BK;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16,
                                                 opb ? blane : alane, (int)so, 0, 0);
      }
    };
    // fragments of one 16-deep k-block (48 VGPRs): B [j][plane], A [i][plane]
    auto read_kb = [&](int buf, int kb, bf16x8g (&fa)[4][2], bf16x8g (&fb)[2][2]) {
      const int c = 2 * kb + h;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = 64 * wn + 32 * j + r;
        const int off = row * GM_BK + 8 * (c ^ ((row >> 2) & 3));
#pragma unroll
        for (int q = 0; q < 2; ++q) fb[j][q] = *reinterpret_cast<const bf16x8g*>(&G.op[buf].b[q][off]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 128 * wm + 32 * i + r;
        const int off = row * GM_BK + 8 * (c ^ ((row >> 2) & 3));
#pragma unroll
        for (int q = 0; q < 2; ++q) fa[i][q] = *reinterpret_cast<const bf16x8g*>(&G.op[buf].a[q][off]);
      }
    };
    auto mfma_kb = [&](const bf16x8g (&fa)[4][2], const bf16x8g (&fb)[2][2]) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma_bf16g(fa[i][1], fb[j][0], acc[i][j]);
          acc[i][j] = mfma_bf16g(fa[i][0], fb[j][1], acc[i][j]);
          acc[i][j] = mfma_bf16g(fa[i][0], fb[j][0], acc[i][j]);
        }
    };
    // two LDS buffers, one barrier per tile, placed between the tile's two
    // k-blocks: behind it tile t + 1 is visible (every wave waited for its own
    // DMA) and every read of tile t's buffer is done (they were issued a
    // barrier earlier), so tile t + 2's DMA goes into that buffer and tile
    // t + 1's fragments are read while k-block 1 of tile t multiplies
    const int nt = K / GM_BK;
    bf16x8g fa0[4][2], fb0[2][2], fa1[4][2], fb1[2][2];
    issue(0, 0);
    __syncthreads();
    if (nt > 1) issue(GM_BK, 1);
    read_kb(0, 0, fa0, fb0);
    read_kb(0, 1, fa1, fb1);
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      mfma_kb(fa0, fb0);
      if (t + 1 < nt) {
        __syncthreads();
        if (t + 2 < nt) issue((t + 2) * GM_BK, buf);
        read_kb(buf ^ 1, 0, fa0, fb0);
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_kb(fa1, fb1);
      if (t + 1 < nt) read_kb(buf ^ 1, 1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // the epilogue's stage overlays the operand buffers
  } else {
  // one register set: tile t + 1 is loaded right after tile t is stored, and
  // the sched_barrier keeps those loads ahead of tile t's MFMAs (at 256 VGPRs
  // the scheduler otherwise sinks them below the MFMAs, where their registers
  // free up, and every store then waits out a full L2 round trip)
  f32x4 ra[4], rb[4];
#if PCADV_GEMM_BIG_DB
  // two LDS buffers, one barrier per tile: tile t + 1 is stored into the
  // other buffer while tile t's MFMAs run (its loads were issued one tile
  // earlier), and tile t + 2's loads go out right after that store
  load_tile(ra, rb, 0);
  store_tile(ra, rb, 0);
  load_tile(ra, rb, GM_BK);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += GM_BK) {
    mfma_tile(buf);
    if (k0 + GM_BK < K) {
      store_tile(ra, rb, buf ^ 1);  // buffer buf ^ 1 was last read before the previous barrier
      load_tile(ra, rb, k0 + 2 * GM_BK);
    }
    __syncthreads();
    buf ^= 1;
  }
#else
  load_tile(ra, rb, 0);
  for (int k0 = 0; k0 < K; k0 += GM_BK) {
    __syncthreads();
    store_tile(ra, rb, 0);
    __syncthreads();
    load_tile(ra, rb, k0 + GM_BK);
    __builtin_amdgcn_sched_barrier(0);
    mfma_tile(0);
  }
#endif
  }

  if constexpr (MODE == 2) {
    // per column, the top-2 (value, row) of this wave's 128 rows: the wave's
    // half of the tile is one 128-row tile of k_max_combine's record
    const int T = 2 * T2;
    const int t128 = 2 * (tx % T2) + wm;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int k1 = GKEY_NONE, k2 = GKEY_NONE;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = 32 * i + acc_row(e, lane);
          if (GL || m0 + 128 * wm + row < Mlim) {  // GL: whole tiles, every row is in range
            const int key = gkey(acc[i][j][e], row);
            k2 = max(min(key, k1), k2);  // median(key, k1, k2) for k2 <= k1
            k1 = max(k1, key);
          }
        }
      const int o1 = __shfl_xor(k1, 32), o2 = __shfl_xor(k2, 32);
      k2 = max(min(k1, o1), max(k2, o2));
      k1 = max(k1, o1);
      const int n = n0 + 64 * wn + 32 * j + r;
      if (h == 0 && n < p.N) p.part[((size_t)cl * T + t128) * p.N + n] = make_int2(k1, k2);
    }
  } else {
    // epilogue through LDS, one 256 x 128 half of the tile at a time (each
    // wave's 32-column block j), rows written by 32 lanes x 4 columns
    float* stage = L.stage;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      __syncthreads();  // the MFMA operands / the previous half are no longer read
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          stage[(128 * wm + 32 * i + acc_row(e, lane)) * GB_ES + 32 * wn + r] = acc[i][j][e];
      __syncthreads();
      const int c4 = 4 * (tid & 31);                 // staged column (0..124)
      const int n = n0 + 64 * (c4 >> 5) + 32 * j + (c4 & 31);
      // 16 rows per thread in batches (the loads of a batch in flight
      // together; the other half's accumulators are still live)
      constexpr int NIT = MODE == 1 ? 2 : 4;  // accumulate: the targets' loads too
      if (MODE == 1 || p.cmask) {
#pragma unroll
        for (int q4 = 0; q4 < 16 / NIT; ++q4)
          epilogue_rows<MODE, NIT>(p, p.c, stage, GB_ES, c4, (tid >> 5) + 16 * NIT * q4, 16, m0, n);
      } else {
        epilogue_rows_plain<MODE>(p, p.c, stage, GB_ES, c4, tid >> 5, 16, 16, m0, n);
      }
    }
  }
}

// diagnostic / A-B switches read from the environment ("1" = on)
static bool getenv_flag(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '1';
}

// the 256-tile kernel takes a plane-operand GEMM when its columns come in
// whole 256-blocks and the grid still gives every CU work (>= 256 tiles);
// PCADV_GEMM_BIG=0 keeps the 128-tile kernel (A/B and bitwise checks)
static bool gemm_big_enabled() {
  const char* e = getenv("PCADV_GEMM_BIG");
  return !(e && e[0] == '0');
}
static bool use_gemm_big(int M, int N, int rows_per_group, int mode, long long lda, long long ldb) {
  if (!gemm_big_enabled() || N % GB_BN != 0) return false;
  // 32-bit buffer offsets (bytes) below 2^31 over the A rows one launch (or
  // one cloud, mode 2) addresses and over B
  if ((long long)(mode == 2 ? rows_per_group : M) * lda * 2 >= 0x7fffffffLL ||
      (long long)N * ldb * 2 >= 0x7fffffffLL)
    return false;
  if (mode == 2 && rows_per_group % GB_BM != 0) return false;
  const long long tiles = (long long)((M + GB_BM - 1) / GB_BM) * (N / GB_BN);
  return tiles >= 256;
}
// LDS-DMA staging for whole tiles (PCADV_GEMM_GLDS=0 keeps register staging:
// same MFMAs in the same order, bitwise the same results)
static bool gemm_glds_enabled() {
  const char* e = getenv("PCADV_GEMM_GLDS");
  return !(e && e[0] == '0');
}
template <int MODE, bool GL>
static int gemm_big_launch_t(const GemmP& p, hipStream_t s) {
  using Lds = typename std::conditional<GL, GemmGlLds, GemmBigLds>::type;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_bf2_big<MODE, GL>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(Lds)) != hipSuccess) {
      set_error("gemm: cannot reserve %zu bytes of LDS", sizeof(Lds));
      return PCADV_EHIP;
    }
    attr = true;
  }
  const dim3 grid((p.M + GB_BM - 1) / GB_BM, p.N / GB_BN, 1);
  hipLaunchKernelGGL((k_gemm_bf2_big<MODE, GL>), grid, dim3(GB_T), sizeof(Lds), s, p);
  PC_HIP_CHECK_LAUNCH("k_gemm_bf2_big");
  return PCADV_OK;
}
template <int MODE>
static int gemm_big_launch(const GemmP& p, hipStream_t s) {
  const bool whole = (MODE == 2 ? p.rows_per_group : p.M) % GB_BM == 0 && p.K % GM_BK == 0;
  return whole && gemm_glds_enabled() ? gemm_big_launch_t<MODE, true>(p, s)
                                      : gemm_big_launch_t<MODE, false>(p, s);
}

// Skinny GEMM (M <= 16 rows per workgroup: one row per cloud, e.g. fc1's
// per-cloud bias gmax W1g^T and the per-cloud gradient s1 W1g) in exact f32
// FMAs on the vector ALUs, with the same epilogue as k_gemm_x3.  The 16 rows
// of A are read by every lane (clamped to the last row, so no per-row
// branches), the reduction axis is spread over the workgroup and combined in a
// fixed order (bitwise reproducible).
//   TB = 0 (B[n][k], k contiguous): a workgroup per column n, 256 lanes
//          across k (16-B loads when aligned);
//   TB = 1 (B[k][n], n contiguous): a workgroup per 16 columns, 16 k-lanes
//          per column.
template <int TB>
__global__ void __launch_bounds__(256)
k_gemm_small(GemmP p) {
  const int tid = threadIdx.x;
  const int m0 = blockIdx.y * 16;
  const int mrows = min(16, p.M - m0);
  const float* arow[16];
#pragma unroll
  for (int mm = 0; mm < 16; ++mm) arow[mm] = p.a + (size_t)(m0 + min(mm, mrows - 1)) * p.lda;
  float acc[16];
#pragma unroll
  for (int mm = 0; mm < 16; ++mm) acc[mm] = 0.f;
  __shared__ float red[16][257];
  int n, part;  // this thread's column and its slot among the column's partial sums
  if (TB == 0) {
    n = blockIdx.x;
    part = tid;
    const float* brow = p.b + (size_t)n * p.ldb;
    if (p.avec && p.bvec) {
      for (int k = 4 * tid; k + 3 < p.K; k += 1024) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(brow + k);
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(arow[mm] + k);
          acc[mm] = fmaf(a[3], b[3], fmaf(a[2], b[2], fmaf(a[1], b[1], fmaf(a[0], b[0], acc[mm]))));
        }
      }
      for (int k = (p.K & ~3) + tid; k < p.K; k += 256) {  // K % 4 tail
        const float b = brow[k];
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) acc[mm] = fmaf(arow[mm][k], b, acc[mm]);
      }
    } else {
      for (int k = tid; k < p.K; k += 256) {
        const float b = brow[k];
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) acc[mm] = fmaf(arow[mm][k], b, acc[mm]);
      }
    }
  } else {
    n = blockIdx.x * 16 + (tid & 15);
    part = tid >> 4;
    if (n < p.N) {
#pragma unroll 4
      for (int k = part; k < p.K; k += 16) {
        const float b = p.b[(size_t)k * p.ldb + n];
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) acc[mm] = fmaf(arow[mm][k], b, acc[mm]);
      }
    }
  }
  // partial sums -> LDS [row][slot], then a fixed-order sum per (row, column)
  const int nslot = TB == 0 ? 256 : 16;
  const int col = TB == 0 ? 0 : (tid & 15);
#pragma unroll
  for (int mm = 0; mm < 16; ++mm) red[mm][TB == 0 ? part : col * 16 + part] = acc[mm];
  __syncthreads();
  int mm, cc;
  if (TB == 0) {
    if (tid >= 16) return;
    mm = tid; cc = 0;
  } else {
    mm = tid >> 4; cc = tid & 15;
    n = blockIdx.x * 16 + cc;
  }
  if (mm >= mrows || n >= p.N) return;
  float v = 0.f;
  const float* src = &red[mm][TB == 0 ? 0 : cc * 16];
  for (int q = 0; q < nslot; ++q) v += src[q];
  const int m = m0 + mm;
  float* dst = p.c + (size_t)m * p.ldc + n;
  v += p.bias ? p.bias[n] : 0.f;
  if (p.bias_rows) v += p.bias_rows[(size_t)(m / p.rows_per_group) * p.N + n];
  if (p.accumulate) v += *dst;
  if (p.relu) v = v > 0.f ? v : 0.f;
  if (p.cmask && !(p.cmask[(size_t)m * p.ldm + n] > 0.f)) v = 0.f;
  *dst = v;
}

// out[g][e] (+)= sum over z < nz of in[(g nz + z) * stride + e], e < E, in a
// fixed order (bitwise reproducible): a workgroup takes 32 consecutive e
// (coalesced) x 8 interleaved z-subsets (one per half-wave), combined through
// LDS.  The output index is 2-D: out + g * ldg + (e / N) * ldo + e % N.
// one z-subset's share (z = zs, zs + 8, ...) of a slab sum, four loads in flight
__device__ __forceinline__ float slab_subset(const float* src, long long stride, int nz, int zs) {
  float s = 0.f;
  int z = zs;
  for (; z + 24 < nz; z += 32) {
    const float a0 = src[(size_t)z * stride], a1 = src[(size_t)(z + 8) * stride];
    const float a2 = src[(size_t)(z + 16) * stride], a3 = src[(size_t)(z + 24) * stride];
    s += ((a0 + a1) + a2) + a3;
  }
  for (; z < nz; z += 8) s += src[(size_t)z * stride];
  return s;
}
// slab_subset on four consecutive elements (16-B loads; the same sums per element)
__device__ __forceinline__ f32x4 slab_subset4(const float* src, long long stride, int nz, int zs) {
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  int z = zs;
  auto ld = [&](int zz) { return *reinterpret_cast<const f32x4*>(src + (size_t)zz * stride); };
  for (; z + 24 < nz; z += 32) {
    const f32x4 a0 = ld(z), a1 = ld(z + 8), a2 = ld(z + 16), a3 = ld(z + 24);
    s += ((a0 + a1) + a2) + a3;
  }
  for (; z < nz; z += 8) s += ld(z);
  return s;
}
// the eight subsets' partials of element el, in subset order
__device__ __forceinline__ float slab_combine(const float (&part)[8][33], int el) {
  float t = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) t += part[q][el];
  return t;
}

__global__ void __launch_bounds__(256)
k_slab_sum(const float* __restrict__ in, long long stride, int nz, long long E,
           float* __restrict__ out, long long ldg, int N, long long ldo, int accumulate) {
  const int tid = threadIdx.x, el = tid & 31, zs = tid >> 5;
  const long long e = (long long)blockIdx.x * 32 + el;
  const int g = blockIdx.y;
  __shared__ float part[8][33];
  part[zs][el] = e < E ? slab_subset(in + (size_t)g * nz * stride + e, stride, nz, zs) : 0.f;
  __syncthreads();
  if (zs == 0 && e < E) {
    const float t = slab_combine(part, el);
    float* dst = out + (size_t)g * ldg + (size_t)(e / N) * ldo + (e % N);
    *dst = accumulate ? *dst + t : t;
  }
}

// The finishing reductions of one weight-gradient launch in ONE launch, bitwise
// the same sums as k_slab_sum's separate launches: blocks [0, nb_dw) sum the dW
// slabs (as k_slab_sum (dw)); the blocks after them take 32 output channels
// each and form the per-group sums of the slabs' column sums (kept in LDS,
// written to gs when asked) and then db from them (or from the column sums
// directly when there is one group and no per-group output).
constexpr int WF_MAXG = 64;
// One weight gradient's finishing reductions (the arguments of k_wgrad_finish)
struct WfDesc {
  const float* slabs; long long E; int nz; float* dw; int N; long long ldo; int acc_dw; int nb_dw;
  const float* csum; int O; int groups; int zpg; int from_groups; float* gs; float* db;
  int acc_db;
};
// dW blocks take WF_DWE consecutive elements (four per thread, 16-B loads when
// the slab stride allows) x the 8 z-subsets; column-sum blocks 32 channels
constexpr int WF_DWE = 128;
struct WfLds {
  float part[8][33];
  float gsl[WF_MAXG][33];
  float pw[8][WF_DWE + 4];
};
__device__ __forceinline__ void wgrad_finish_block(const WfDesc& w, int blk, WfLds& L) {
  float (&part)[8][33] = L.part;
  float (&gsl)[WF_MAXG][33] = L.gsl;
  const float* __restrict__ slabs = w.slabs;
  const long long E = w.E;
  const int nz = w.nz, N = w.N, acc_dw = w.acc_dw, nb_dw = w.nb_dw, O = w.O, groups = w.groups;
  const int zpg = w.zpg, from_groups = w.from_groups, acc_db = w.acc_db;
  const long long ldo = w.ldo;
  float* __restrict__ dw = w.dw;
  const float* __restrict__ csum = w.csum;
  float* __restrict__ gs = w.gs;
  float* __restrict__ db = w.db;
  const int tid = threadIdx.x, el = tid & 31, zs = tid >> 5;
  if (blk < nb_dw) {
    const long long e0 = (long long)blk * WF_DWE + 4 * el;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (E % 4 == 0) {
      if (e0 < E) v = slab_subset4(slabs + e0, E, nz, zs);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (e0 + t < E) v[t] = slab_subset(slabs + e0 + t, E, nz, zs);
    }
    *reinterpret_cast<f32x4*>(&L.pw[zs][4 * el]) = v;
    __syncthreads();
    // thread tid < 128 finishes element blk * 128 + tid (coalesced stores)
    const long long e = (long long)blk * WF_DWE + tid;
    if (tid < WF_DWE && e < E) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) t += L.pw[q][tid];
      float* dst = dw + (size_t)(e / N) * ldo + (e % N);
      *dst = acc_dw ? *dst + t : t;
    }
    return;
  }
  const int o = (blk - nb_dw) * 32 + el;
  const bool ok = o < O;
  if (!from_groups) {
    part[zs][el] = ok ? slab_subset(csum + o, O, nz, zs) : 0.f;
    __syncthreads();
    if (zs == 0 && ok) {
      const float t = slab_combine(part, el);
      db[o] = acc_db ? db[o] + t : t;
    }
    return;
  }
  for (int g = 0; g < groups; ++g) {
    part[zs][el] = ok ? slab_subset(csum + (size_t)g * zpg * O + o, O, zpg, zs) : 0.f;
    __syncthreads();
    if (zs == 0) {
      const float t = slab_combine(part, el);
      gsl[g][el] = t;
      if (gs && ok) gs[(size_t)g * O + o] = t;
    }
    __syncthreads();
  }
  if (!db) return;
  // db over the groups: the same subset order, reading the group sums from LDS
  {
    float s = 0.f;
    int z = zs;
    for (; z + 24 < groups; z += 32) s += ((gsl[z][el] + gsl[z + 8][el]) + gsl[z + 16][el]) + gsl[z + 24][el];
    for (; z < groups; z += 8) s += gsl[z][el];
    part[zs][el] = ok ? s : 0.f;
  }
  __syncthreads();
  if (zs == 0 && ok) {
    const float t = slab_combine(part, el);
    db[o] = acc_db ? db[o] + t : t;
  }
}

__global__ void __launch_bounds__(256)
k_wgrad_finish(const float* __restrict__ slabs, long long E, int nz, float* __restrict__ dw, int N,
               long long ldo, int acc_dw, int nb_dw, const float* __restrict__ csum, int O,
               int groups, int zpg, int from_groups, float* __restrict__ gs, float* __restrict__ db,
               int acc_db) {
  __shared__ WfLds L;
  const WfDesc w{slabs, E, nz, dw, N, ldo, acc_dw, nb_dw, csum, O, groups, zpg, from_groups, gs, db,
                 acc_db};
  wgrad_finish_block(w, (int)blockIdx.x, L);
}

// Several weight gradients' finishing reductions in one launch
// (launch_wgrad_finish, after their launch_gemm_wgrad_slabs calls): block b belongs
// to the descriptor whose block range [blk0[i], blk0[i + 1]) holds it; every
// sum is bitwise the one k_wgrad_finish forms.
constexpr int WF_BATCH = 16;
struct WfBatch {
  WfDesc d[WF_BATCH];
  int blk0[WF_BATCH + 1];
  int n;
};
__global__ void __launch_bounds__(256)
k_wgrad_finish_batch(WfBatch bt) {
  __shared__ WfLds L;
  const int b = (int)blockIdx.x;
  int i = 0;
  for (int j = 1; j < bt.n; ++j) i = b >= bt.blk0[j] ? j : i;
  wgrad_finish_block(bt.d[i], b - bt.blk0[i], L);
}

// column sums of an M x N matrix (row stride ld), optionally masked by [Y > 0]
// (Y stored alike): bias gradients.  One workgroup per 64 columns x row chunk,
// partial sums in fixed order, then a second pass over the chunks.
__global__ void __launch_bounds__(256)
k_colsum_part(const float* __restrict__ x, const float* __restrict__ ymask, long long ld,
              long long ldm, int M, int N, int rows_per_chunk, float* __restrict__ part) {
  const int c0 = blockIdx.x * 64, chunk = blockIdx.y;
  const int col = c0 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  __shared__ float sm[4][64];
  float s = 0.f;
  if (col < N) {
    const int r0 = chunk * rows_per_chunk, r1 = min(M, r0 + rows_per_chunk);
    for (int m = r0 + rg; m < r1; m += 4) {
      const float v = x[(size_t)m * ld + col];
      s += (!ymask || ymask[(size_t)m * ldm + col] > 0.f) ? v : 0.f;
    }
  }
  sm[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && col < N)
    part[(size_t)chunk * N + col] = ((sm[0][threadIdx.x] + sm[1][threadIdx.x]) + sm[2][threadIdx.x]) +
                                    sm[3][threadIdx.x];
}

__global__ void __launch_bounds__(256)
k_colsum_fin(const float* __restrict__ part, int nchunk, int N, float* __restrict__ out,
             int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int c = 0; c < nchunk; ++c) s += part[(size_t)c * N + n];
  out[n] = accumulate ? out[n] + s : s;
}

// ---------------------------------------------------------------------------
// max over points after a screened GEMM: merge the per-tile top-2 keys of each
// (cloud, channel), re-evaluate the winner and the runner-up as exact f32 dot
// products of the input row with the weight row, rank them by those, then apply
// the bias and the ReLU before the max (pointnet.py:301-303: relu(conv6) then
// torch.max).  Eight lanes per row (octet DPP sums), as k_conv4_max's tail.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dppg(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float octet_sum_g(float v) {
  v += dppg<0xB1>(v);
  v += dppg<0x4E>(v);
  v += dppg<0x141>(v);
  return v;
}

__device__ __forceinline__ bool rank_before_g(float va, int ia, float vb, int ib) {
  const bool na = va != va, nb = vb != vb;
  if (na || nb) return na && (!nb || ia < ib);
  return va > vb || (va == vb && ia < ib);
}
__device__ __forceinline__ float gkey_value(int k) {
  const int ord = k & ~127;
  return __int_as_float(ord ^ ((ord >> 31) & 0x7fffffff));
}

// one wave per 8 (cloud, channel) pairs; x rows [C*Npts][K] (row stride ldx)
__global__ void __launch_bounds__(256)
k_max_combine(const int2* __restrict__ part, int T, int Npts, int C, int O,
              const float* __restrict__ x, long long ldx, int K, const float* __restrict__ w,
              const float* __restrict__ bias, int relu, float* __restrict__ gmax,
              int32_t* __restrict__ gidx) {
  const int lane = threadIdx.x & 63;
  const int pair = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (lane >> 3);
  const int part_lane = lane & 7;
  const bool valid = pair < C * O;
  const int c = valid ? pair / O : 0, o = valid ? pair % O : 0;
  float v1 = -INFINITY, v2 = -INFINITY;
  int i1 = 0x7fffffff, i2 = 0x7fffffff;
  if (valid) {
    for (int t = part_lane; t < T; t += 8) {  // tiles of this cloud: rows t*128 ..
      const int2 kk = part[(size_t)(c * T + t) * O + o];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int key = q ? kk.y : kk.x;
        if (key == GKEY_NONE) continue;
        const float v = gkey_value(key);
        const int idx = t * GM_BM + 127 - (key & 127);
        const bool a = rank_before_g(v, idx, v1, i1);
        const bool b = !a && rank_before_g(v, idx, v2, i2);
        const float nv2 = a ? v1 : (b ? v : v2);
        const int ni2 = a ? i1 : (b ? idx : i2);
        v1 = a ? v : v1;
        i1 = a ? idx : i1;
        v2 = nv2;
        i2 = ni2;
      }
    }
  }
  // merge the octet's lists (xor 1, 2, 4 within the octet)
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    const float a1 = __shfl_xor(v1, m), a2 = __shfl_xor(v2, m);
    const int j1 = __shfl_xor(i1, m), j2 = __shfl_xor(i2, m);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float v = q ? a2 : a1;
      const int idx = q ? j2 : j1;
      const bool a = rank_before_g(v, idx, v1, i1);
      const bool b = !a && rank_before_g(v, idx, v2, i2);
      const float nv2 = a ? v1 : (b ? v : v2);
      const int ni2 = a ? i1 : (b ? idx : i2);
      v1 = a ? v : v1;
      i1 = a ? idx : i1;
      v2 = nv2;
      i2 = ni2;
    }
  }
  if (i1 == 0x7fffffff) i1 = 0;
  // both screened candidates are re-evaluated exactly and ranked by the exact
  // values (the screening error scales with sum |x w|, not with the pooled
  // value: no window on the screened gap is safe; see k_conv4_max)
  const bool near = i2 != 0x7fffffff;
  const int j2 = near ? i2 : i1;
  // exact dots: lane part_lane of the octet takes terms part_lane*4 + 32 u
  const float* xr1 = x + (size_t)(c * Npts + i1) * ldx;
  const float* xr2 = x + (size_t)(c * Npts + j2) * ldx;
  const float* wr = w + (size_t)o * K;
  float e1 = 0.f, e2 = 0.f;
  if (valid) {
    for (int k = 4 * part_lane; k < K; k += 32) {
      const f32x4 wv = *reinterpret_cast<const f32x4*>(wr + k);
      const f32x4 a = *reinterpret_cast<const f32x4*>(xr1 + k);
      const f32x4 b = *reinterpret_cast<const f32x4*>(xr2 + k);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        e1 = fmaf(a[t], wv[t], e1);
        e2 = fmaf(b[t], wv[t], e2);
      }
    }
  }
  e1 = octet_sum_g(e1);
  e2 = octet_sum_g(e2);
  if (valid && part_lane == 0) {
    const float bb = bias ? bias[o] : 0.f;
    e1 += bb;
    e2 += bb;
    const bool second = near && rank_before_g(e2, i2, e1, i1);
    float g = second ? e2 : e1;
    if (relu) g = g > 0.f ? g : 0.f;
    gmax[(size_t)c * O + o] = g;
    gidx[(size_t)c * O + o] = second ? i2 : i1;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// the engine's loads are buffer loads with 32-bit byte offsets from the
// operand base (a masked element reads at 2^31): every operand must span < 2^31 B
static bool fits31(long long rows, long long ld, int esz) {
  return rows >= 0 && ld >= 0 && (rows * ld + 16) * esz < 0x7fffffffLL;
}

template <typename K>
static int gemm_lds_attr(K kern, size_t bytes = sizeof(GemmLds)) {
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
    set_error("gemm: cannot reserve %zu bytes of LDS", bytes);
    return PCADV_EHIP;
  }
  return PCADV_OK;
}

// LDS of k_gemm_x3: the register-staged tile, or (VEC bit 2) two LDS-DMA
// buffers of 4 plane tiles of 128 x 32 bf16
template <int VEC>
constexpr size_t gemm_x3_lds_bytes() {
  return (VEC & 4) ? (sizeof(GemmLds) > 65536 ? sizeof(GemmLds) : 65536) : sizeof(GemmLds);
}

template <int TA, int TB, int MODE, int NP, int VEC>
static int gemm_launch_direct(const GemmP& p, dim3 grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    PC_TRY_GEMM(gemm_lds_attr(k_gemm_x3<TA, TB, MODE, NP, VEC>, gemm_x3_lds_bytes<VEC>()));
    attr = true;
  }
  hipLaunchKernelGGL((k_gemm_x3<TA, TB, MODE, NP, VEC>), grid, dim3(GM_T), gemm_x3_lds_bytes<VEC>(), s, p);
  PC_HIP_CHECK_LAUNCH("k_gemm_x3");
  return PCADV_OK;
}

// Pairing inside ONE call (pcadv_gemm_wgrad_slabs): a slot on the caller's
// stack.  With slot->on, the first pairable weight-gradient or data-gradient
// GEMM waits in the slot; the next one of the other kind launches both as one
// k_gemm_x3_pair; gemm_slot_flush enqueues a GEMM still waiting.  Nothing
// outlives the call.
struct PendingGemm {
  bool on, has;
  int kind;  // 0: weight gradient <1, 1, 0, 6, v>; 1: data gradient <0, 1, mode, np, v>
  int v, mode, np;
  GemmP p;
  dim3 grid;
};

static PairGeom pair_geom(dim3 g) {
  return PairGeom{(int)(g.x * g.y * g.z), (int)g.x, (int)g.y, (int)g.z};
}

static int gemm_slot_flush(PendingGemm& slot, hipStream_t s) {
  if (!slot.has) return PCADV_OK;
  slot.has = false;
  const GemmP& p = slot.p;
  const dim3 g = slot.grid;
  if (slot.kind == 0) {
    switch (slot.v) {
      case 1: return gemm_launch_direct<1, 1, 0, 6, 1>(p, g, s);
      case 2: return gemm_launch_direct<1, 1, 0, 6, 2>(p, g, s);
      default: return gemm_launch_direct<1, 1, 0, 6, 3>(p, g, s);
    }
  }
  if (slot.np == 6) {
    if (slot.mode == 0)
      return slot.v == 2 ? gemm_launch_direct<0, 1, 0, 6, 2>(p, g, s)
                         : gemm_launch_direct<0, 1, 0, 6, 3>(p, g, s);
    return slot.v == 2 ? gemm_launch_direct<0, 1, 1, 6, 2>(p, g, s)
                       : gemm_launch_direct<0, 1, 1, 6, 3>(p, g, s);
  }
  if (slot.mode == 0)
    return slot.v == 2 ? gemm_launch_direct<0, 1, 0, 3, 2>(p, g, s)
                       : gemm_launch_direct<0, 1, 0, 3, 3>(p, g, s);
  return slot.v == 2 ? gemm_launch_direct<0, 1, 1, 3, 2>(p, g, s)
                     : gemm_launch_direct<0, 1, 1, 3, 3>(p, g, s);
}

// which GEMM's workgroups a pair dispatches first: the weight gradient's
// (its slab workgroups run the longest; A/B on two boxes 1.139 -> 1.125 and
// 1.182 -> 1.167 ms against the issue order); PCADV_PAIR_WFIRST=0: the data
// gradient's, =i: the GEMM issued first.  Outputs bitwise the same either way.
static int pair_wfirst(int issued) {
  static const int v = [] {
    const char* e = getenv("PCADV_PAIR_WFIRST");
    if (e && e[0] == '0') return 0;
    if (e && e[0] == 'i') return -1;
    return 1;
  }();
  return v < 0 ? issued : v;
}
template <int VW, int MD, int VD, int NPD>
static int gemm_pair_launch(const GemmP& pw, dim3 gw, const GemmP& pd, dim3 gd, int wfirst,
                            hipStream_t s) {
  wfirst = pair_wfirst(wfirst);
  static bool attr = false;
  if (!attr) {
    PC_TRY_GEMM(gemm_lds_attr(k_gemm_x3_pair<VW, MD, VD, NPD>));
    attr = true;
  }
  const PairGeom a = pair_geom(gw), b = pair_geom(gd);
  hipLaunchKernelGGL((k_gemm_x3_pair<VW, MD, VD, NPD>), dim3((unsigned)(a.n + b.n)), dim3(GM_T),
                     sizeof(GemmLds), s, pw, a, pd, b, wfirst);
  PC_HIP_CHECK_LAUNCH("k_gemm_x3_pair");
  return PCADV_OK;
}

template <int TA, int TB, int MODE, int NP, int VEC>
static int gemm_launch_v(const GemmP& p, dim3 grid, hipStream_t s, PendingGemm* slot) {
  constexpr bool is_w = TA == 1 && TB == 1 && MODE == 0 && NP == 6 && VEC >= 1;
  constexpr bool is_d = TA == 0 && TB == 1 && (MODE == 0 || MODE == 1) && VEC >= 2;
  if constexpr (is_w || is_d) {
    if (slot && slot->on) {
      if (slot->has && slot->kind == (is_w ? 1 : 0)) {  // the pair's second GEMM
        slot->has = false;
        if constexpr (is_w) {
          const GemmP& pd = slot->p;
          const dim3 gd = slot->grid;
          if (slot->np == 6) {
            if (slot->mode == 0)
              return slot->v == 2 ? gemm_pair_launch<VEC, 0, 2, 6>(p, grid, pd, gd, 0, s)
                                  : gemm_pair_launch<VEC, 0, 3, 6>(p, grid, pd, gd, 0, s);
            return slot->v == 2 ? gemm_pair_launch<VEC, 1, 2, 6>(p, grid, pd, gd, 0, s)
                                : gemm_pair_launch<VEC, 1, 3, 6>(p, grid, pd, gd, 0, s);
          }
          if (slot->mode == 0)
            return slot->v == 2 ? gemm_pair_launch<VEC, 0, 2, 3>(p, grid, pd, gd, 0, s)
                                : gemm_pair_launch<VEC, 0, 3, 3>(p, grid, pd, gd, 0, s);
          return slot->v == 2 ? gemm_pair_launch<VEC, 1, 2, 3>(p, grid, pd, gd, 0, s)
                              : gemm_pair_launch<VEC, 1, 3, 3>(p, grid, pd, gd, 0, s);
        } else {
          const GemmP& pw = slot->p;
          const dim3 gw = slot->grid;
          switch (slot->v) {
            case 1: return gemm_pair_launch<1, MODE, VEC, NP>(pw, gw, p, grid, 1, s);
            case 2: return gemm_pair_launch<2, MODE, VEC, NP>(pw, gw, p, grid, 1, s);
            default: return gemm_pair_launch<3, MODE, VEC, NP>(pw, gw, p, grid, 1, s);
          }
        }
      }
      PC_TRY_GEMM(gemm_slot_flush(*slot, s));  // a waiting GEMM of the same kind goes alone
      slot->has = true;
      slot->kind = is_w ? 0 : 1;
      slot->v = VEC;
      slot->mode = MODE;
      slot->np = NP;
      slot->p = p;
      slot->grid = grid;
      return PCADV_OK;
    }
  }
  return gemm_launch_direct<TA, TB, MODE, NP, VEC>(p, grid, s);
}

// the staging form of each operand: 16-byte loads where the operand allows
// them (aligned, row stride % 4) and no vector straddles an edge (rows: the
// reduction range [kz0, kz1) in multiples of 4; columns: M or N % 4), else dwords
template <int TA, int TB>
static int gemm_vec_flags(const GemmP& p) {
  const bool kq = p.K % 4 == 0 && p.grp % 4 == 0 && (p.zpg == 1 || p.ksplit_len % 4 == 0);
  const bool va = TA == 2 || (p.avec && (TA == 0 ? kq : p.M % 4 == 0 && p.rows_per_group % 4 == 0));
  const bool vb = TB >= 2 || (p.bvec && (TB == 0 ? kq : p.N % 4 == 0));
  return (va ? 1 : 0) | (vb ? 2 : 0);
}

template <int TA, int TB, int MODE, int NP>
static int gemm_launch_grid(const GemmP& p, dim3 grid, hipStream_t s, PendingGemm* slot) {
  switch (gemm_vec_flags<TA, TB>(p)) {
    case 3: return gemm_launch_v<TA, TB, MODE, NP, 3>(p, grid, s, slot);
    case 2: return gemm_launch_v<TA, TB, MODE, NP, 2>(p, grid, s, slot);
    case 1: return gemm_launch_v<TA, TB, MODE, NP, 1>(p, grid, s, slot);
    default: return gemm_launch_v<TA, TB, MODE, NP, 0>(p, grid, s, slot);
  }
}
template <int TA, int TB, int MODE, int NP>
static int gemm_launch(const GemmP& p, int nz, hipStream_t s, PendingGemm* slot = nullptr) {
  return gemm_launch_grid<TA, TB, MODE, NP>(
      p, dim3((p.M + GM_BM - 1) / GM_BM, (p.N + GM_BN - 1) / GM_BN, nz), s, slot);
}

// C[M][N] (+)= op(A) op(B)^T: see the header comment for ta / tb.
static int launch_gemm_impl(const float* a, long long lda, int ta, const float* b, long long ldb,
                            int tb, float* c, long long ldc, int M, int N, int K,
                            const float* bias, const float* bias_rows, int rows_per_group,
                            int relu, int accumulate, const float* cmask, long long ldm,
                            int precise, void* c_hi, void* c_lo, long long ldcp, hipStream_t s,
                            PendingGemm* slot) {
  PC_REQUIRE(a && b && c && M > 0 && N > 0 && K > 0, "gemm: bad shape M=%d N=%d K=%d", M, N, K);
  PC_REQUIRE((ta == 0 && lda >= K) || (ta == 1 && lda >= M), "gemm: bad lda %lld (ta=%d)", lda, ta);
  PC_REQUIRE((tb == 0 && ldb >= K) || (tb == 1 && ldb >= N), "gemm: bad ldb %lld (tb=%d)", ldb, tb);
  PC_REQUIRE(((uintptr_t)a & 3) == 0 && ((uintptr_t)b & 3) == 0 && ((uintptr_t)c & 3) == 0,
             "gemm: operands must be float aligned");
  PC_REQUIRE(ldc >= N, "gemm: bad ldc %lld", ldc);
  PC_REQUIRE(!cmask || ldm >= N, "gemm: bad ldm %lld", ldm);
  PC_REQUIRE(!bias_rows || rows_per_group > 0, "gemm: bias_rows needs rows_per_group");
  PC_REQUIRE(ta == 0 || tb == 1, "gemm: A^T needs B^T (the weight-gradient form)");
  PC_REQUIRE(fits31(ta ? K : M, lda, 4) && fits31(tb ? K : N, ldb, 4) && fits31(M, ldc, 4) &&
                 (!cmask || fits31(M, ldm, 4)),
             "gemm: operands must span < 2 GB (M=%d N=%d K=%d)", M, N, K);
  GemmP p{};
  p.a = a; p.lda = lda; p.b = b; p.ldb = ldb; p.c = c; p.ldc = ldc;
  p.cmask = cmask; p.ldm = ldm;
  p.bias = bias; p.bias_rows = bias_rows; p.rows_per_group = rows_per_group;
  p.M = M; p.N = N; p.K = K; p.relu = relu; p.accumulate = accumulate;
  p.avec = lda % 4 == 0 && ((uintptr_t)a & 15) == 0;
  p.bvec = ldb % 4 == 0 && ((uintptr_t)b & 15) == 0;
  p.cvec = ldc % 4 == 0 && ((uintptr_t)c & 15) == 0 && (!bias || ((uintptr_t)bias & 15) == 0) &&
           (!bias_rows || (N % 4 == 0 && ((uintptr_t)bias_rows & 15) == 0)) &&
           (!cmask || (ldm % 4 == 0 && ((uintptr_t)cmask & 15) == 0));
  p.grp = K; p.zpg = 1; p.ksplit_len = K;
  PC_REQUIRE(!c_hi == !c_lo && (!c_hi || (ldcp >= N && ldcp % 4 == 0 && N % 4 == 0 && p.cvec &&
                                         ((uintptr_t)c_hi & 7) == 0 && ((uintptr_t)c_lo & 7) == 0)),
             "gemm: output planes need N %% 4, ldcp %% 4 and 16-B aligned C");
  p.cp[0] = static_cast<__bf16*>(c_hi); p.cp[1] = static_cast<__bf16*>(c_lo); p.ldcp = ldcp;
  PC_REQUIRE(!c_hi || !(ta == 0 && M <= 32), "gemm: output planes need M > 32");
  if (ta == 0 && M <= 32) {  // per-cloud rows: exact f32 on the vector ALUs
    const dim3 grid(tb ? (N + 15) / 16 : N, (M + 15) / 16);
    if (tb) hipLaunchKernelGGL(k_gemm_small<1>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_gemm_small<0>, grid, dim3(256), 0, s, p);
    PC_HIP_CHECK_LAUNCH("k_gemm_small");
    return PCADV_OK;
  }
  if (precise) {
    if (ta == 0 && tb == 0) return accumulate ? gemm_launch<0, 0, 1, 6>(p, 1, s) : gemm_launch<0, 0, 0, 6>(p, 1, s);
    if (ta == 0 && tb == 1)
      return accumulate ? gemm_launch<0, 1, 1, 6>(p, 1, s, slot) : gemm_launch<0, 1, 0, 6>(p, 1, s, slot);
    return accumulate ? gemm_launch<1, 1, 1, 6>(p, 1, s) : gemm_launch<1, 1, 0, 6>(p, 1, s);
  }
  if (ta == 0 && tb == 0) return accumulate ? gemm_launch<0, 0, 1, 3>(p, 1, s) : gemm_launch<0, 0, 0, 3>(p, 1, s);
  if (ta == 0 && tb == 1)
    return accumulate ? gemm_launch<0, 1, 1, 3>(p, 1, s, slot) : gemm_launch<0, 1, 0, 3>(p, 1, s, slot);
  return accumulate ? gemm_launch<1, 1, 1, 3>(p, 1, s) : gemm_launch<1, 1, 0, 3>(p, 1, s);
}

int launch_gemm(const float* a, long long lda, int ta, const float* b, long long ldb, int tb,
                float* c, long long ldc, int M, int N, int K, const float* bias,
                const float* bias_rows, int rows_per_group, int relu, int accumulate,
                const float* cmask, long long ldm, int precise, void* c_hi, void* c_lo,
                long long ldcp, hipStream_t s) {
  return launch_gemm_impl(a, lda, ta, b, ldb, tb, c, ldc, M, N, K, bias, bias_rows, rows_per_group,
                          relu, accumulate, cmask, ldm, precise, c_hi, c_lo, ldcp, s, nullptr);
}

// Both operands as bf16 hi / lo planes (the 2-way splits of f32 matrices, made
// once by their producers): the three-product forward GEMM with no per-tile
// splitting; C (f32) and optionally C's own planes for the next layer.
int launch_gemm_bf2(const void* a_hi, const void* a_lo, long long lda, const void* b_hi,
                    const void* b_lo, long long ldb, float* c, long long ldc, void* c_hi,
                    void* c_lo, long long ldcp, int M, int N, int K, const float* bias,
                    const float* bias_rows, int rows_per_group, int relu, int accumulate,
                    const float* cmask, long long ldm, hipStream_t s) {
  PC_REQUIRE(a_hi && a_lo && b_hi && b_lo && c && M > 0 && N > 0 && K > 0,
             "gemm_bf2: bad shape M=%d N=%d K=%d", M, N, K);
  PC_REQUIRE(K % 16 == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K,
             "gemm_bf2: K %% 16 and lda, ldb %% 8 required (K=%d lda=%lld ldb=%lld)", K, lda, ldb);
  PC_REQUIRE((((uintptr_t)a_hi | (uintptr_t)a_lo | (uintptr_t)b_hi | (uintptr_t)b_lo) & 15) == 0,
             "gemm_bf2: planes must be 16-B aligned");
  PC_REQUIRE(ldc >= N && (!cmask || ldm >= N) && (!bias_rows || rows_per_group > 0),
             "gemm_bf2: bad ldc / ldm / bias_rows");
  PC_REQUIRE(fits31(M, lda, 2) && fits31(N, ldb, 2) && fits31(M, ldc, 4) &&
                 (!cmask || fits31(M, ldm, 4)),
             "gemm_bf2: operands must span < 2 GB");
  GemmP p{};
  p.ap[0] = static_cast<const __bf16*>(a_hi); p.ap[1] = static_cast<const __bf16*>(a_lo);
  p.ldap = lda;
  p.bp[0] = static_cast<const __bf16*>(b_hi); p.bp[1] = static_cast<const __bf16*>(b_lo);
  p.ldbp = ldb;
  p.c = c; p.ldc = ldc; p.cmask = cmask; p.ldm = ldm;
  p.bias = bias; p.bias_rows = bias_rows; p.rows_per_group = rows_per_group;
  p.M = M; p.N = N; p.K = K; p.relu = relu; p.accumulate = accumulate;
  p.cvec = ldc % 4 == 0 && ((uintptr_t)c & 15) == 0 && (!bias || ((uintptr_t)bias & 15) == 0) &&
           (!bias_rows || (N % 4 == 0 && ((uintptr_t)bias_rows & 15) == 0)) &&
           (!cmask || (ldm % 4 == 0 && ((uintptr_t)cmask & 15) == 0));
  PC_REQUIRE(!c_hi == !c_lo && (!c_hi || (ldcp >= N && ldcp % 4 == 0 && N % 4 == 0 && p.cvec)),
             "gemm_bf2: output planes need N %% 4, ldcp %% 4 and 16-B aligned C");
  p.cp[0] = static_cast<__bf16*>(c_hi); p.cp[1] = static_cast<__bf16*>(c_lo); p.ldcp = ldcp;
  p.grp = K; p.zpg = 1; p.ksplit_len = K;
  // whole 128-tiles: the LDS-DMA 128-tile kernel, also where the 256-tile one
  // would apply (conv5: 1.1211 -> 1.1180 ms A/B, two workgroups per CU over
  // four k-tiles beat one); PCADV_GEMM_BIG_PLAIN=1 keeps the 256 tiles there
  const bool gl128 = M % GM_BM == 0 && N % GM_BN == 0 && K % GM_BK == 0 && gemm_glds_enabled();
  if ((!gl128 || getenv_flag("PCADV_GEMM_BIG_PLAIN")) && use_gemm_big(M, N, 0, 0, lda, ldb))
    return accumulate ? gemm_big_launch<1>(p, s) : gemm_big_launch<0>(p, s);
  if (gl128) {
    const dim3 grid(M / GM_BM, N / GM_BN, 1);
    return accumulate ? gemm_launch_direct<2, 2, 1, 3, 7>(p, grid, s)
                      : gemm_launch_direct<2, 2, 0, 3, 7>(p, grid, s);
  }
  return accumulate ? gemm_launch<2, 2, 1, 3>(p, 1, s) : gemm_launch<2, 2, 0, 3>(p, 1, s);
}

// f32 [rows][cols] (row stride ld) -> bf16 hi / lo planes (row stride ldo)
__global__ void __launch_bounds__(256)
k_split_bf2(const float* __restrict__ x, long long ld, int rows, int cols, __bf16* __restrict__ hi,
            __bf16* __restrict__ lo, long long ldo) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)rows * cols) return;
  const int r = (int)(e / cols), c = (int)(e % cols);
  const float v = x[(size_t)r * ld + c];
  const __bf16 h = (__bf16)v;
  hi[(size_t)r * ldo + c] = h;
  lo[(size_t)r * ldo + c] = (__bf16)(v - (float)h);
}

int launch_split_bf2(const float* x, long long ld, int rows, int cols, void* hi, void* lo,
                     long long ldo, hipStream_t s) {
  PC_REQUIRE(x && hi && lo && rows > 0 && cols > 0 && ld >= cols && ldo >= cols,
             "split_bf2: bad arguments");
  const long long n = (long long)rows * cols;
  hipLaunchKernelGGL(k_split_bf2, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ld, rows,
                     cols, static_cast<__bf16*>(hi), static_cast<__bf16*>(lo), ldo);
  PC_HIP_CHECK_LAUNCH("k_split_bf2");
  return PCADV_OK;
}

// f32 [rows][cols] -> bf16 hi / mid / lo planes (split_planes<3>: bitwise the
// three-way split the six-product GEMMs make of an f32 operand per tile); hi and
// mid are also the two-way split's hi / lo (split_planes<2>)
__global__ void __launch_bounds__(256)
k_split_bf3(const float* __restrict__ x, long long ld, int rows, int cols, __bf16* __restrict__ hi,
            __bf16* __restrict__ mid, __bf16* __restrict__ lo, long long ldo) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)rows * cols) return;
  const int r = (int)(e / cols), c = (int)(e % cols);
  __bf16 o[3];
  split_planes<3>(x[(size_t)r * ld + c], o);
  const size_t d = (size_t)r * ldo + c;
  hi[d] = o[0];
  mid[d] = o[1];
  lo[d] = o[2];
}

int launch_split_bf3(const float* x, long long ld, int rows, int cols, void* hi, void* mid,
                     void* lo, long long ldo, hipStream_t s) {
  PC_REQUIRE(x && hi && mid && lo && rows > 0 && cols > 0 && ld >= cols && ldo >= cols,
             "split_bf3: bad arguments");
  const long long n = (long long)rows * cols;
  hipLaunchKernelGGL(k_split_bf3, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ld, rows,
                     cols, static_cast<__bf16*>(hi), static_cast<__bf16*>(mid),
                     static_cast<__bf16*>(lo), ldo);
  PC_HIP_CHECK_LAUNCH("k_split_bf3");
  return PCADV_OK;
}

// The six-product GEMM C[M][N] (+)= A B^T with A f32 [m][k] (split three ways
// per tile, as launch_gemm with precise = 1, ta = tb = 0) and B given as the
// hi / mid / lo planes of its three-way split ([n][k], made once by
// pcadv_split_bf3): the same MFMAs on the same values, so C is bitwise
// launch_gemm's, without B's per-tile VALU split.
int launch_gemm_b3(const float* a, long long lda, const void* b_hi, const void* b_mid,
                   const void* b_lo, long long ldb, float* c, long long ldc, int M, int N, int K,
                   const float* bias, const float* bias_rows, int rows_per_group, int relu,
                   int accumulate, hipStream_t s) {
  PC_REQUIRE(a && b_hi && b_mid && b_lo && c && M > 32 && N > 0 && K > 0,
             "gemm_b3: bad shape M=%d N=%d K=%d (M > 32)", M, N, K);
  PC_REQUIRE(K % 16 == 0 && ldb % 8 == 0 && ldb >= K && lda >= K,
             "gemm_b3: K %% 16 and ldb %% 8 required (K=%d ldb=%lld)", K, ldb);
  PC_REQUIRE((((uintptr_t)b_hi | (uintptr_t)b_mid | (uintptr_t)b_lo) & 15) == 0,
             "gemm_b3: planes must be 16-B aligned");
  PC_REQUIRE(((uintptr_t)a & 3) == 0 && ((uintptr_t)c & 3) == 0, "gemm_b3: float alignment");
  PC_REQUIRE(ldc >= N && (!bias_rows || rows_per_group > 0), "gemm_b3: bad ldc / bias_rows");
  PC_REQUIRE(fits31(M, lda, 4) && fits31(N, ldb, 2) && fits31(M, ldc, 4),
             "gemm_b3: operands must span < 2 GB");
  GemmP p{};
  p.a = a; p.lda = lda;
  p.bp[0] = static_cast<const __bf16*>(b_hi); p.bp[1] = static_cast<const __bf16*>(b_mid);
  p.bp[2] = static_cast<const __bf16*>(b_lo); p.ldbp = ldb;
  p.c = c; p.ldc = ldc;
  p.bias = bias; p.bias_rows = bias_rows; p.rows_per_group = rows_per_group;
  p.M = M; p.N = N; p.K = K; p.relu = relu; p.accumulate = accumulate;
  p.avec = lda % 4 == 0 && ((uintptr_t)a & 15) == 0;
  p.bvec = 1;
  p.cvec = ldc % 4 == 0 && ((uintptr_t)c & 15) == 0 && (!bias || ((uintptr_t)bias & 15) == 0) &&
           (!bias_rows || (N % 4 == 0 && ((uintptr_t)bias_rows & 15) == 0));
  p.grp = K; p.zpg = 1; p.ksplit_len = K;
  return accumulate ? gemm_launch<0, 3, 1, 6>(p, 1, s) : gemm_launch<0, 3, 0, 6>(p, 1, s);
}

// weight gradient dW[O][Kin] (+)= sum over the rows of dZ[row][o] X[row][k]:
// A = dZ^T (stored [rows][O], row stride ldz), B = X^T (stored [rows][Kin],
// ldx); the row axis is cut into fixed-order slabs (zpg per group of
// rows_per_group rows, or of all rows) reduced by k_slab_sum, which also
// forms db[o] (+)= sum dZ[.][o] and the per-group sums gsum[g][o] from the
// column sums the slabs take of the staged dZ.  Enough slabs to give the
// launch ~768 workgroups, each slab at least 128 rows.
#ifndef PCADV_WGRAD_WGS
#define PCADV_WGRAD_WGS 512  // one dispatch round (two 61 KB-LDS workgroups per CU)
#endif
#ifndef PCADV_WGRAD_FLOOR
#define PCADV_WGRAD_FLOOR 0
#endif
struct WgradPlan { int groups, grp, zpg, len, nz; };
// the workgroups a weight gradient's slab plan aims at (PCADV_WGRAD_WGS
// overrides the default, read once: the workspace size follows the plan)
static int wgrad_wgs() {
  static const int v = [] {
    const char* e = getenv("PCADV_WGRAD_WGS");
    const int x = e ? atoi(e) : 0;
    return x > 0 ? x : PCADV_WGRAD_WGS;
  }();
  return v;
}
static WgradPlan wgrad_plan(int rows, int O, int Kin, int rows_per_group) {
  WgradPlan w{};
  w.grp = rows_per_group > 0 ? rows_per_group : rows;
  w.groups = rows / w.grp;
  const int tiles = ((O + GM_BM - 1) / GM_BM) * ((Kin + GM_BN - 1) / GM_BN);
#if PCADV_WGRAD_FLOOR
  const int want = max(1, wgrad_wgs() / (tiles * w.groups));
#else
  const int want = (wgrad_wgs() + tiles * w.groups - 1) / (tiles * w.groups);
#endif
  w.zpg = max(1, min(want, (w.grp + 127) / 128));
  w.len = (w.grp + w.zpg - 1) / w.zpg;
  w.zpg = (w.grp + w.len - 1) / w.len;
  w.nz = w.groups * w.zpg;
  return w;
}

size_t gemm_wgrad_workspace_bytes(int rows, int O, int Kin, int rows_per_group) {
  if (rows <= 0 || O <= 0 || Kin <= 0 || (rows_per_group > 0 && rows % rows_per_group)) return 0;
  const WgradPlan w = wgrad_plan(rows, O, Kin, rows_per_group);
  return ((size_t)w.nz * O * Kin + (size_t)w.nz * O + (size_t)w.groups * O) * sizeof(float) + 512;
}

// Weight gradients over a few rows (fc1's tiled global columns: the B
// per-cloud sums s[b][o] times gmax / the class vector, pointnet.py:306-310):
// dw[o][k] (+)= sum_{b < B} s[b][o] x[b][k] in exact f32, b in order (fixed,
// deterministic), four k per thread; up to two x operands (jobs) per launch,
// blocks [0, nb0) on job 0.  Replaces a six-product slab GEMM over B = 16
// rows (one k-tile of work on a 128 x 128 tile engine).
struct WsmJob { const float* x; long long ldx; int K; float* dw; };
__global__ void __launch_bounds__(256)
k_wgrad_small(const float* __restrict__ s, long long lds, int B, int O, long long ldo, int accumulate,
              WsmJob j0, WsmJob j1, int nb0) {
  const bool second = (int)blockIdx.x >= nb0;
  const WsmJob j = second ? j1 : j0;
  const int blk = second ? (int)blockIdx.x - nb0 : (int)blockIdx.x;
  const int kq = (j.K + 3) / 4;  // k quads per output row
  const long long e = (long long)blk * 256 + threadIdx.x;
  if (e >= (long long)O * kq) return;
  const int o = (int)(e / kq), k = 4 * (int)(e % kq);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (int b = 0; b < B; ++b) {
    const float sv = s[(size_t)b * lds + o];
    const float* xr = j.x + (size_t)b * j.ldx + k;
    a0 = fmaf(sv, xr[0], a0);
    if (k + 1 < j.K) a1 = fmaf(sv, xr[1], a1);
    if (k + 2 < j.K) a2 = fmaf(sv, xr[2], a2);
    if (k + 3 < j.K) a3 = fmaf(sv, xr[3], a3);
  }
  float* d = j.dw + (size_t)o * ldo + k;
  const float r[4] = {a0, a1, a2, a3};
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (k + t < j.K) d[t] = accumulate ? d[t] + r[t] : r[t];
}

int launch_wgrad_small(const float* s, long long lds, int B, int O, const float* x0, long long ldx0,
                       int K0, float* dw0, const float* x1, long long ldx1, int K1, float* dw1,
                       long long ldo, int accumulate, hipStream_t st) {
  PC_REQUIRE(s && x0 && dw0 && B > 0 && O > 0 && K0 > 0 && lds >= O && ldx0 >= K0 && ldo >= K0 &&
                 (!x1 || (dw1 && K1 > 0 && ldx1 >= K1 && ldo >= K1)),
             "wgrad_small: bad shape B=%d O=%d K0=%d K1=%d", B, O, K0, K1);
  const long long n0 = (long long)O * ((K0 + 3) / 4), n1 = x1 ? (long long)O * ((K1 + 3) / 4) : 0;
  const int nb0 = (int)((n0 + 255) / 256), nb1 = (int)((n1 + 255) / 256);
  const WsmJob j0{x0, ldx0, K0, dw0};
  const WsmJob j1{x1 ? x1 : x0, x1 ? ldx1 : ldx0, x1 ? K1 : K0, x1 ? dw1 : dw0};
  hipLaunchKernelGGL(k_wgrad_small, dim3((unsigned)(nb0 + nb1)), dim3(256), 0, st, s, lds, B, O,
                     ldo, accumulate, j0, j1, nb0);
  PC_HIP_CHECK_LAUNCH("k_wgrad_small");
  return PCADV_OK;
}

// A weight gradient's slab GEMM: its plan, its GemmP and the slab / column-sum
// regions of its workspace (shared by the one-call and the split forms)
struct WgradJob {
  WgradPlan w;
  GemmP p;
  float* slabs;
  float* csum;
  long long E;
};
static int wgrad_prepare(const float* dz, long long ldz, const float* x, long long ldx, int rows,
                         int O, int Kin, float* dw, long long ldo, float* db, float* gsum,
                         int rows_per_group, void* ws, size_t ws_bytes, WgradJob& j) {
  PC_REQUIRE(dz && x && dw && rows > 0 && O > 0 && Kin > 0 && ldo >= Kin && ldz >= O && ldx >= Kin,
             "gemm_wgrad: bad shape rows=%d O=%d Kin=%d", rows, O, Kin);
  PC_REQUIRE(!gsum || (rows_per_group > 0 && rows % rows_per_group == 0),
             "gemm_wgrad: per-group sums need rows %% rows_per_group == 0");
  PC_REQUIRE(fits31(rows, ldz, 4) && fits31(rows, ldx, 4), "gemm_wgrad: operands must span < 2 GB");
  PC_REQUIRE(rows_per_group <= 0 || rows % rows_per_group == 0, "gemm_wgrad: rows %% rows_per_group");
  j.w = wgrad_plan(rows, O, Kin, rows_per_group);
  PC_REQUIRE(ws && ws_bytes >= gemm_wgrad_workspace_bytes(rows, O, Kin, rows_per_group),
             "gemm_wgrad: workspace");
  j.slabs = static_cast<float*>(ws);
  j.csum = (db || gsum) ? j.slabs + (size_t)j.w.nz * O * Kin : nullptr;
  GemmP& p = j.p;
  p = GemmP{};
  p.a = dz; p.lda = ldz; p.b = x; p.ldb = ldx;
  p.c = j.slabs; p.ldc = Kin;
  p.M = O; p.N = Kin; p.K = rows;
  p.avec = ldz % 4 == 0 && ((uintptr_t)dz & 15) == 0;
  p.bvec = ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
  p.cvec = Kin % 4 == 0;
  p.grp = j.w.grp; p.zpg = j.w.zpg; p.ksplit_len = j.w.len;
  p.slab_stride = (long long)O * Kin;
  p.csum = j.csum;
  j.E = (long long)O * Kin;
  return PCADV_OK;
}

// the per-group sums (gsum, or the workspace's scratch rows) of the slabs'
// column sums and db from them, by separate k_slab_sum launches: the form for
// more groups than k_wgrad_finish keeps in LDS
static int wgrad_colsums_split(const WgradJob& j, int O, float* db, float* gsum, int accumulate,
                               hipStream_t s) {
  const bool from_groups = j.w.groups > 1 || gsum;
  float* gs = gsum ? gsum : j.csum + (size_t)j.w.nz * O;
  if (from_groups) {
    hipLaunchKernelGGL(k_slab_sum, dim3((O + 31) / 32, j.w.groups), dim3(256), 0, s,
                       static_cast<const float*>(j.csum), (long long)O, j.w.zpg, (long long)O, gs,
                       (long long)O, O, 0LL, 0);
    PC_HIP_CHECK_LAUNCH("k_slab_sum (groups)");
  }
  if (db) {
    hipLaunchKernelGGL(k_slab_sum, dim3((O + 31) / 32, 1), dim3(256), 0, s,
                       static_cast<const float*>(from_groups ? gs : j.csum), (long long)O,
                       from_groups ? j.w.groups : j.w.nz, (long long)O, db, 0LL, O, 0LL,
                       accumulate);
    PC_HIP_CHECK_LAUNCH("k_slab_sum (db)");
  }
  return PCADV_OK;
}

int launch_gemm_wgrad(const float* dz, long long ldz, const float* x, long long ldx, int rows,
                      int O, int Kin, float* dw, long long ldo, float* db, float* gsum,
                      int rows_per_group, int accumulate, void* ws, size_t ws_bytes, hipStream_t s) {
  WgradJob j;
  PC_TRY_GEMM(wgrad_prepare(dz, ldz, x, ldx, rows, O, Kin, dw, ldo, db, gsum, rows_per_group, ws,
                            ws_bytes, j));
  PC_TRY_GEMM((gemm_launch<1, 1, 0, 6>(j.p, j.w.nz, s)));
  const WgradPlan& w = j.w;
  const long long E = j.E;
  float* slabs = j.slabs;
  float* csum = j.csum;
  if (w.groups <= WF_MAXG && !getenv_flag("PCADV_WGRAD_SPLIT_FINISH")) {
    // dW, the per-group sums and db in one launch (k_wgrad_finish)
    const int nb_dw = (int)((E + WF_DWE - 1) / WF_DWE);
    const int nb_cs = csum ? (O + 31) / 32 : 0;
    const bool from_groups = w.groups > 1 || gsum;
    hipLaunchKernelGGL(k_wgrad_finish, dim3((unsigned)(nb_dw + nb_cs)), dim3(256), 0, s,
                       static_cast<const float*>(slabs), E, w.nz, dw, Kin, ldo, accumulate, nb_dw,
                       static_cast<const float*>(csum), O, w.groups, w.zpg, from_groups ? 1 : 0,
                       gsum, db, accumulate);
    PC_HIP_CHECK_LAUNCH("k_wgrad_finish");
    return PCADV_OK;
  }
  hipLaunchKernelGGL(k_slab_sum, dim3((unsigned)((E + 31) / 32), 1), dim3(256), 0, s,
                     static_cast<const float*>(slabs), E, w.nz, E, dw, 0LL, Kin, ldo, accumulate);
  PC_HIP_CHECK_LAUNCH("k_slab_sum (dw)");
  if (csum) PC_TRY_GEMM(wgrad_colsums_split(j, O, db, gsum, accumulate, s));
  return PCADV_OK;
}

static int wgrad_prepare_d(const pcadv_wgrad_desc& d, WgradJob& j) {
  return wgrad_prepare(d.dz, d.ldz, d.x, d.ldx, d.rows, d.O, d.Kin, d.dw, d.ldo, d.db, d.gsum,
                       d.rows_per_group, d.workspace, d.workspace_bytes, j);
}

// The slab GEMM of w (+ gsum and its db now, when asked) and optionally the
// data-gradient GEMM g, paired into one launch where both forms allow it.
// The dw (and db) sums are left to launch_wgrad_finish.
int launch_gemm_wgrad_slabs(const pcadv_wgrad_desc* wd, const pcadv_gemm_desc* g, hipStream_t s) {
  PC_REQUIRE(wd, "gemm_wgrad_slabs: null descriptor");
  const pcadv_wgrad_desc& d = *wd;
  WgradJob j;
  PC_TRY_GEMM(wgrad_prepare_d(d, j));
  PendingGemm slot{};
  slot.on = g != nullptr;
  PC_TRY_GEMM((gemm_launch<1, 1, 0, 6>(j.p, j.w.nz, s, &slot)));
  if (g)
    PC_TRY_GEMM(launch_gemm_impl(g->a, g->lda, g->ta, g->b, g->ldb, g->tb, g->c, g->ldc, g->M, g->N,
                                 g->K, g->bias, g->bias_rows, g->rows_per_group, g->relu,
                                 g->accumulate, g->cmask, g->ldm, g->precise, g->c_hi, g->c_lo,
                                 g->ldcp, s, &slot));
  PC_TRY_GEMM(gemm_slot_flush(slot, s));  // a GEMM that found no partner goes alone
  if (d.gsum) {  // fc1's per-cloud sums are needed at once: finish the column sums now
    if (j.w.groups <= WF_MAXG) {
      hipLaunchKernelGGL(k_wgrad_finish, dim3((unsigned)((d.O + 31) / 32)), dim3(256), 0, s,
                         static_cast<const float*>(j.slabs), j.E, j.w.nz, d.dw, d.Kin, d.ldo,
                         d.accumulate, 0, static_cast<const float*>(j.csum), d.O, j.w.groups,
                         j.w.zpg, 1, d.gsum, d.db, d.accumulate);
      PC_HIP_CHECK_LAUNCH("k_wgrad_finish (groups)");
    } else {
      PC_TRY_GEMM(wgrad_colsums_split(j, d.O, d.db, d.gsum, d.accumulate, s));
    }
  }
  return PCADV_OK;
}

// The finishing sums of n weight gradients whose slabs launch_gemm_wgrad_slabs
// enqueued: one k_wgrad_finish_batch launch per WF_BATCH descriptors, bitwise
// the sums of launch_gemm_wgrad.  Column sums over more groups than the batch
// kernel keeps in LDS take the separate k_slab_sum form.
int launch_wgrad_finish(const pcadv_wgrad_desc* ds, int n, hipStream_t s) {
  PC_REQUIRE(n >= 0 && (ds || n == 0), "wgrad_finish: bad descriptor list (n=%d)", n);
  WfBatch b{};
  auto flush = [&]() -> int {
    if (b.n == 0) return PCADV_OK;
    hipLaunchKernelGGL(k_wgrad_finish_batch, dim3((unsigned)b.blk0[b.n]), dim3(256), 0, s, b);
    PC_HIP_CHECK_LAUNCH("k_wgrad_finish_batch");
    b.n = 0;
    b.blk0[0] = 0;
    return PCADV_OK;
  };
  for (int i = 0; i < n; ++i) {
    const pcadv_wgrad_desc& d = ds[i];
    WgradJob j;
    PC_TRY_GEMM(wgrad_prepare_d(d, j));
    const int nb_dw = (int)((j.E + WF_DWE - 1) / WF_DWE);
    const bool from_groups = j.w.groups > 1 || d.gsum;
    // gsum's column sums (and db) were finished by the slabs call
    const bool cs = j.csum && !d.gsum;
    const bool cs_here = cs && !(from_groups && j.w.groups > WF_MAXG);
    if (cs && !cs_here) PC_TRY_GEMM(wgrad_colsums_split(j, d.O, d.db, nullptr, d.accumulate, s));
    const int nb_cs = cs_here ? (d.O + 31) / 32 : 0;
    const WfDesc w{j.slabs, j.E, j.w.nz, d.dw, d.Kin, d.ldo, d.accumulate, nb_dw,
                   cs_here ? j.csum : nullptr, d.O, j.w.groups, j.w.zpg, from_groups ? 1 : 0,
                   nullptr, cs_here ? d.db : nullptr, d.accumulate};
    if (b.n == WF_BATCH) PC_TRY_GEMM(flush());
    b.d[b.n] = w;
    b.blk0[b.n + 1] = b.blk0[b.n] + nb_dw + nb_cs;
    ++b.n;
  }
  return flush();
}

constexpr int CS_ROWS = 128;  // rows per colsum chunk (enough workgroups to fill the chip)

size_t colsum_workspace_bytes(int M, int N) {
  const int nchunk = (M + CS_ROWS - 1) / CS_ROWS;
  return (size_t)nchunk * N * sizeof(float) + 256;
}

// per-group column sums: out[g][n] = sum over rows g*rpg .. of x[m][n] (* [Y > 0])
int launch_group_colsum(const float* x, const float* ymask, long long ld, long long ldm, int M,
                        int N, int rows_per_group, float* out, hipStream_t s) {
  PC_REQUIRE(x && out && M > 0 && N > 0 && rows_per_group > 0 && M % rows_per_group == 0,
             "group_colsum: bad shape");
  hipLaunchKernelGGL(k_colsum_part, dim3((N + 63) / 64, M / rows_per_group), dim3(256), 0, s, x,
                     ymask, ld, ldm, M, N, rows_per_group, out);
  PC_HIP_CHECK_LAUNCH("k_colsum_part");
  return PCADV_OK;
}

int launch_colsum(const float* x, const float* ymask, long long ld, long long ldm, int M, int N,
                  float* out, int accumulate, void* ws, size_t ws_bytes, hipStream_t s) {
  PC_REQUIRE(x && out && M > 0 && N > 0, "colsum: bad shape");
  const int nchunk = (M + CS_ROWS - 1) / CS_ROWS;
  PC_REQUIRE(ws && ws_bytes >= colsum_workspace_bytes(M, N), "colsum: workspace");
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(k_colsum_part, dim3((N + 63) / 64, nchunk), dim3(256), 0, s, x, ymask, ld,
                     ldm, M, N, CS_ROWS, part);
  PC_HIP_CHECK_LAUNCH("k_colsum_part");
  hipLaunchKernelGGL(k_colsum_fin, dim3((N + 255) / 256), dim3(256), 0, s, part, nchunk, N, out,
                     accumulate);
  PC_HIP_CHECK_LAUNCH("k_colsum_fin");
  return PCADV_OK;
}

// gmax[c][o] = max over the Npts points of cloud c of act(x w^T + b), gidx its
// argmax: a screened GEMM (per 128-row tile top-2) then k_max_combine.
size_t conv_max_x3_workspace_bytes(int C, int Npts, int O) {
  const int T = (Npts + GM_BM - 1) / GM_BM;
  return (size_t)C * T * O * sizeof(int2) + 256;
}

int launch_conv_max_x3(const float* x, long long ldx, int C, int Npts, int K, const float* w,
                       const float* b, int O, int relu, float* gmax, int32_t* gidx, void* ws,
                       size_t ws_bytes, hipStream_t s, const void* x_hi = nullptr,
                       const void* x_lo = nullptr, long long ldxp = 0, const void* w_hi = nullptr,
                       const void* w_lo = nullptr) {
  PC_REQUIRE(x && w && gmax && gidx && C > 0 && Npts > 0 && K > 0 && O > 0,
             "conv_max_x3: bad shape");
  PC_REQUIRE(K % 32 == 0 && ldx % 4 == 0, "conv_max_x3: K %% 32 and ldx %% 4 required");
  PC_REQUIRE(ws && ws_bytes >= conv_max_x3_workspace_bytes(C, Npts, O), "conv_max_x3: workspace");
  PC_REQUIRE(fits31(Npts, ldx, 4) && fits31(Npts, ldxp, 2) && fits31(O, K, 4),
             "conv_max_x3: a cloud's rows and the weights must span < 2 GB");
  const bool planes = x_hi != nullptr;
  PC_REQUIRE(!planes || (x_lo && w_hi && w_lo && ldxp % 8 == 0 && ldxp >= K &&
                         ((((uintptr_t)x_hi | (uintptr_t)x_lo | (uintptr_t)w_hi | (uintptr_t)w_lo) & 15) == 0)),
             "conv_max_x3: planes need ldxp %% 8 and 16-B alignment");
  const int T = (Npts + GM_BM - 1) / GM_BM;
  int2* part = static_cast<int2*>(ws);
  {
    GemmP p{};
    p.a = x; p.lda = ldx; p.b = w; p.ldb = K;
    p.c = gmax; p.ldc = O;
    p.avec = ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
    p.bvec = K % 4 == 0 && ((uintptr_t)w & 15) == 0;
    if (planes) {
      p.ap[0] = static_cast<const __bf16*>(x_hi); p.ap[1] = static_cast<const __bf16*>(x_lo);
      p.ldap = ldxp;
      p.bp[0] = static_cast<const __bf16*>(w_hi); p.bp[1] = static_cast<const __bf16*>(w_lo);
      p.ldbp = K;
    }
    p.rows_per_group = Npts;
    p.M = C * Npts; p.N = O; p.K = K; p.grp = K; p.zpg = 1; p.ksplit_len = K;
    p.part = part;
    const dim3 grid(C * T, (O + GM_BN - 1) / GM_BN, 1);
    if (planes && use_gemm_big(C * Npts, O, Npts, 2, ldxp, K)) {
      PC_TRY_GEMM(gemm_big_launch<2>(p, s));
    } else if (planes) {
      PC_TRY_GEMM((gemm_launch_grid<2, 2, 2, 3>(p, grid, s, nullptr)));
    } else {
      PC_TRY_GEMM((gemm_launch_grid<0, 0, 2, 3>(p, grid, s, nullptr)));
    }
  }
  const int pairs = C * O;
  hipLaunchKernelGGL(k_max_combine, dim3((pairs + 31) / 32), dim3(256), 0, s, part, T, Npts, C, O,
                     x, ldx, K, w, b, relu, gmax, gidx);
  PC_HIP_CHECK_LAUNCH("k_max_combine");
  return PCADV_OK;
}


// ---------------------------------------------------------------------------
// CrossEntropyLoss over rows (pointnet/train_pointnet_seg.py:152 applied at
// utils/trainer.py:344 to pred (B, C, N) vs seg (B, N): the mean over all B*N
// points): loss and dL/dlogits * scale, logits point-major [M][Ccls].
// One wave per 64 rows (a lane per row); per-block partial losses, summed in a
// fixed order by the last launch.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_row_ce(const float* __restrict__ logits, long long ld, const int64_t* __restrict__ labels, int M,
         int Ccls, float scale, float* __restrict__ dlogits, float* __restrict__ part) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  float l = 0.f;
  if (m < M) {
    const float* x = logits + (size_t)m * ld;
    float mx = -INFINITY;
    for (int c = 0; c < Ccls; ++c) mx = fmaxf(mx, x[c]);
    float se = 0.f;
    for (int c = 0; c < Ccls; ++c) se += expf(x[c] - mx);
    const float lse = mx + logf(se);
    const int64_t y = labels[m];
    l = lse - x[y];
    const float inv = scale / (float)M;
    float* d = dlogits + (size_t)m * ld;
    for (int c = 0; c < Ccls; ++c) d[c] = (expf(x[c] - lse) - (c == y ? 1.f : 0.f)) * inv;
  }
  __shared__ float sm[256];
  sm[threadIdx.x] = l;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sm[threadIdx.x] += sm[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sm[0];
}

// The same per row, with the block's rows staged through LDS: the logits come
// in and the gradients go out as coalesced rows (a lane per row walking its
// own row touched a new cache line per load: 64 lines per wave instruction).
// Each row's max, exp sum and gradient follow the lane-per-row order above,
// so the results are the same.  LDS rows padded to an odd stride.
constexpr int CE_MAXC = 63;  // the staged rows stay within the default 64 KB of LDS
__global__ void __launch_bounds__(256)
k_row_ce_lds(const float* __restrict__ logits, long long ld, const int64_t* __restrict__ labels,
             int M, int Ccls, float scale, float* __restrict__ dlogits, float* __restrict__ part,
             float* __restrict__ loss) {
  extern __shared__ float xs[];  // [256][Ccls | 1]
  const int S = Ccls | 1, tid = threadIdx.x, r0 = blockIdx.x * 256;
  const int nrows = min(256, M - r0), ne = nrows * Ccls;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(logits), (short)0, 0x7fffffff, 0x00020000);
  // element e = tid + 256 i of the block's rows: (row, col) stepped without divisions
  const int q256 = 256 / Ccls, r256 = 256 % Ccls;
  {
    int row = tid / Ccls, col = tid % Ccls;
    for (int e0 = 0; e0 < ne; e0 += 256 * 8) {
      float v[8];
      int rw[8], cl[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bool ok = e0 + tid + 256 * i < ne;
        uint32_t off = ok ? (uint32_t)(((long long)(r0 + row) * ld + col) * 4) : 0x80000000u;
        asm("" : "+v"(off));
        v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
        rw[i] = row;
        cl[i] = col;
        row += q256;
        col += r256;
        if (col >= Ccls) {
          col -= Ccls;
          ++row;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (e0 + tid + 256 * i < ne) xs[rw[i] * S + cl[i]] = v[i];
    }
  }
  const int m = r0 + tid;
  const int64_t y = m < M ? labels[m] : 0;
  __syncthreads();
  float l = 0.f;
  if (tid < nrows) {
    float* x = xs + tid * S;
    float mx = -INFINITY;
    for (int c = 0; c < Ccls; ++c) mx = fmaxf(mx, x[c]);
    float se = 0.f;
    for (int c = 0; c < Ccls; ++c) se += expf(x[c] - mx);
    const float lse = mx + logf(se);
    l = lse - x[y];
    const float inv = scale / (float)M;
    for (int c = 0; c < Ccls; ++c) x[c] = (expf(x[c] - lse) - (c == y ? 1.f : 0.f)) * inv;
  }
  __syncthreads();
  {
    int row = tid / Ccls, col = tid % Ccls;
    for (int e = tid; e < ne; e += 256) {
      dlogits[(size_t)(r0 + row) * ld + col] = xs[row * S + col];
      row += q256;
      col += r256;
      if (col >= Ccls) {
        col -= Ccls;
        ++row;
      }
    }
  }
  __shared__ float sm[256];
  sm[tid] = l;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) sm[tid] += sm[tid + w];
    __syncthreads();
  }
  if (tid == 0) {
    part[blockIdx.x] = sm[0];
    // one block (M <= 256, the classification heads): the mean here, as
    // k_row_ce_fin forms it, and no finishing launch
    if (gridDim.x == 1) *loss = (float)((double)sm[0] / (double)M);
  }
}

// Few rows (M <= 256, Ccls <= 64: the classification heads' CE over a batch):
// one wave per row, the lanes across the classes, wave butterflies for the max
// and the exp sum (a lane walking its row serially left 32 active lanes in a
// 40-step dependent chain, three times); the batch mean in row order.
__global__ void __launch_bounds__(1024)
k_row_ce_wave(const float* __restrict__ logits, long long ld, const int64_t* __restrict__ labels,
              int M, int Ccls, float scale, float* __restrict__ dlogits, float* __restrict__ loss) {
  __shared__ float rl[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const float inv = scale / (float)M;
  for (int m = wave; m < M; m += nw) {
    const float* x = logits + (size_t)m * ld;
    const int y = (int)labels[m];
    const float v = lane < Ccls ? x[lane] : -INFINITY;
    float mx = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float e = lane < Ccls ? expf(v - mx) : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o);
    const float lse = mx + logf(e);
    if (lane < Ccls)
      dlogits[(size_t)m * ld + lane] = (expf(v - lse) - (lane == y ? 1.f : 0.f)) * inv;
    const float xy = __shfl(v, y);
    if (lane == 0) rl[m] = lse - xy;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int m = 0; m < M; ++m) s += rl[m];
    *loss = (float)(s / (double)M);
  }
}

__global__ void k_row_ce_fin(const float* __restrict__ part, int nb, int M, float* __restrict__ loss) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[b];
  *loss = (float)(s / (double)M);
}

size_t row_ce_workspace_bytes(int M) { return (size_t)((M + 255) / 256) * sizeof(float) + 256; }

int launch_row_ce(const float* logits, long long ld, const int64_t* labels, int M, int Ccls,
                  float scale, float* loss, float* dlogits, void* ws, size_t ws_bytes,
                  hipStream_t s) {
  PC_REQUIRE(logits && labels && loss && dlogits && M > 0 && Ccls > 0 && ld >= Ccls,
             "row_ce: bad shape");
  PC_REQUIRE(ws && ws_bytes >= row_ce_workspace_bytes(M), "row_ce: workspace");
  PC_REQUIRE((long long)M * ld * 4 < 0x7fffffffLL, "row_ce: logits must span < 2 GB");
  const int nb = (M + 255) / 256;
  float* part = static_cast<float*>(ws);
  if (M <= 256 && Ccls <= 64) {
    hipLaunchKernelGGL(k_row_ce_wave, dim3(1), dim3(1024), 0, s, logits, ld, labels, M, Ccls,
                       scale, dlogits, loss);
    PC_HIP_CHECK_LAUNCH("k_row_ce_wave");
    return PCADV_OK;
  }
  if (Ccls <= CE_MAXC) {
    hipLaunchKernelGGL(k_row_ce_lds, dim3(nb), dim3(256), 256 * (Ccls | 1) * sizeof(float), s,
                       logits, ld, labels, M, Ccls, scale, dlogits, part, loss);
    PC_HIP_CHECK_LAUNCH("k_row_ce");
    if (nb == 1) return PCADV_OK;  // the block wrote the mean
  } else {
    hipLaunchKernelGGL(k_row_ce, dim3(nb), dim3(256), 0, s, logits, ld, labels, M, Ccls, scale,
                       dlogits, part);
    PC_HIP_CHECK_LAUNCH("k_row_ce");
  }
  hipLaunchKernelGGL(k_row_ce_fin, dim3(1), dim3(64), 0, s, part, nb, M, loss);
  PC_HIP_CHECK_LAUNCH("k_row_ce_fin");
  return PCADV_OK;
}

// ---------------------------------------------------------------------------
// Backward of relu(x w^T + b) then max over points (pointnet.py:301-303): the
// gradient g[c][o] of the pooled value reaches only the argmax point, and only
// when the max is positive (relu'):  g' = g [gmax > 0]
//   dW[o][k] = sum_c g'[c][o] x[c, gidx[c][o], k],   db[o] = sum_c g'[c][o]
//   dX[c, p, :] += sum_{o: gidx[c][o] = p} g'[c][o] W[o, :]   (in increasing o)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(128)
k_cmx_dw(const float* __restrict__ g, const float* __restrict__ gmax,
         const int32_t* __restrict__ gidx, const float* __restrict__ x, long long ldx, int C,
         int Npts, int O, int K, float* __restrict__ dw, float* __restrict__ db) {
  const int o = blockIdx.x, k = blockIdx.y * 512 + threadIdx.x * 4;  // 4 columns per thread
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float sb = 0.f;
  // CB clouds' gradients, argmax rows and x rows in flight at once (a cloud at
  // a time was two dependent round trips each), summed in cloud order; a zero
  // g' is skipped as before (0 * an infinite x would be a NaN)
  constexpr int CB = 8;
  const int kk = min(k, K - 4);
  for (int c0 = 0; c0 < C; c0 += CB) {
    float gv[CB];
    int gi[CB];
    f32x4 v[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const size_t co = (size_t)min(c0 + u, C - 1) * O + o;
      gv[u] = (c0 + u < C && gmax[co] > 0.f) ? g[co] : 0.f;
      gi[u] = gidx[co];
    }
#pragma unroll
    for (int u = 0; u < CB; ++u)
      v[u] = *reinterpret_cast<const f32x4*>(x + (size_t)(min(c0 + u, C - 1) * Npts + gi[u]) * ldx + kk);
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      sb += gv[u];
      if (gv[u] == 0.f || k >= K) continue;
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = fmaf(gv[u], v[u][t], acc[t]);
    }
  }
  if (k < K) *reinterpret_cast<f32x4*>(dw + (size_t)o * K + k) = acc;
  if (blockIdx.y == 0 && threadIdx.x == 0 && db) db[o] = sb;
}

// One workgroup (8 waves) per (64-point range, cloud).  The cloud's live hits
// (g' != 0) whose argmax falls in the range are marked in a per-point bit set
// over the channels (LDS atomicOr: order-free), flattened into one list sorted
// by (point, o) (popcount prefixes), and the list is cut into 8 equal pieces,
// one per wave, so a point that wins hundreds of channels (a hull point) is
// spread over the waves instead of serialising one.  A wave walks its piece
// with its lanes across the K columns (4 per lane per 256), eight hits' loads
// in flight, and writes a point when the point changes; a point cut by a piece
// boundary is finished by the wave that holds its first hit, adding the later
// waves' partial sums in wave order.  Fixed summation order: bitwise
// reproducible.  relu_x: the additions are masked by [x > 0] at (point,
// column), the relu' of the layer that produced x (x = relu(previous conv)).
constexpr int CMX_PTS = 64, CMX_MAXO = 4096, CMX_MAXK = 512, CMX_W = 8, CMX_U = 8;
constexpr int CMX_T = CMX_MAXK / 256;  // f32x4 column groups per lane
struct CmxLds {
  unsigned bits[CMX_PTS][CMX_MAXO / 32];
  int start[CMX_PTS + 1];
  int list[CMX_MAXO];                 // (point in range) << 16 | o, sorted
  float carry[CMX_W][CMX_MAXK];       // a wave's partial sum of the point it starts inside
  int carry_pt[CMX_W];
};

__global__ void __launch_bounds__(CMX_W * 64)
k_cmx_dx(const float* __restrict__ g, const float* __restrict__ gmax,
         const int32_t* __restrict__ gidx, int Npts, int O, int K, const float* __restrict__ w,
         const float* __restrict__ x, long long ldx, int relu_x, float* __restrict__ dx,
         long long lddx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  CmxLds& L = *reinterpret_cast<CmxLds*>(smem);
  const int c = blockIdx.y, p0 = blockIdx.x * CMX_PTS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nw = (O + 31) / 32;
  for (int i = tid; i < CMX_PTS * nw; i += CMX_W * 64) L.bits[i / nw][i % nw] = 0u;
  __syncthreads();
  for (int o = tid; o < O; o += CMX_W * 64) {
    const size_t co = (size_t)c * O + o;
    if (gmax[co] > 0.f && g[co] != 0.f) {
      const int pl = gidx[co] - p0;
      if (pl >= 0 && pl < CMX_PTS) atomicOr(&L.bits[pl][o >> 5], 1u << (o & 31));
    }
  }
  __syncthreads();
  // hits per point (wave 0, a lane per point), exclusive scan -> start[]
  if (wave == 0) {
    int cnt = 0;
    for (int i = 0; i < nw; ++i) cnt += __popc(L.bits[lane][i]);
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    L.start[lane] = incl - cnt;
    if (lane == 63) L.start[CMX_PTS] = incl;
  }
  __syncthreads();
  // flatten: wave w lists the points w, w + 8, ... (their o in increasing order)
  for (int pl = wave; pl < CMX_PTS; pl += CMX_W) {
    int pos0 = L.start[pl];
    for (int w0 = 0; w0 < nw; w0 += 64) {
      const unsigned word = w0 + lane < nw ? L.bits[pl][w0 + lane] : 0u;
      const int cnt = __popc(word);
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      int pos = pos0 + incl - cnt;
      for (unsigned bw = word; bw; bw &= bw - 1)
        L.list[pos++] = (pl << 16) | ((w0 + lane) * 32 + __builtin_ctz(bw));
      pos0 += __shfl(incl, 63);
    }
  }
  if (tid < CMX_W) L.carry_pt[tid] = -1;
  __syncthreads();
  const int H = L.start[CMX_PTS];
  const int chunk = (H + CMX_W - 1) / CMX_W;
  const int lo = min(H, wave * chunk), hi = min(H, lo + chunk);
  const bool has = lo < hi;
  const int lead = has ? L.list[lo] >> 16 : -1;
  const bool lead_cut = has && lo > 0 && (L.list[lo - 1] >> 16) == lead;  // started in an earlier piece
  const bool tail_cut = has && hi < H && (L.list[hi] >> 16) == (L.list[hi - 1] >> 16);  // continues
  f32x4 acc[CMX_T];
#pragma unroll
  for (int t = 0; t < CMX_T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto write_point = [&](int pl) {  // dx[point] += acc (masked), or hand acc on as a carry
    if (pl == lead && lead_cut) {
#pragma unroll
      for (int t = 0; t < CMX_T; ++t)
        *reinterpret_cast<f32x4*>(&L.carry[wave][256 * t + 4 * lane]) = acc[t];
      if (lane == 0) L.carry_pt[wave] = pl;
      return;
    }
    const size_t row = (size_t)c * Npts + p0 + pl;
#pragma unroll
    for (int t = 0; t < CMX_T; ++t) {
      const int col = 256 * t + 4 * lane;
      if (col >= K) continue;
      f32x4* d = reinterpret_cast<f32x4*>(dx + row * lddx + col);
      f32x4 v = *d, a = acc[t];
      if (relu_x) {
        const f32x4 xv = *reinterpret_cast<const f32x4*>(x + row * ldx + col);
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = xv[u] > 0.f ? a[u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] += a[u];
      *d = v;
    }
  };
  int cur = lead;
  for (int i0 = lo; i0 < hi; i0 += CMX_U) {
    int e[CMX_U];
    float gv[CMX_U];
    f32x4 wv[CMX_U][CMX_T];
#pragma unroll
    for (int u = 0; u < CMX_U; ++u) {  // every load of the group first
      const int i = min(i0 + u, hi - 1);
      e[u] = L.list[i];
      const int o = e[u] & 0xffff;
      gv[u] = i0 + u < hi ? g[(size_t)c * O + o] : 0.f;
#pragma unroll
      for (int t = 0; t < CMX_T; ++t) {
        const int col = min(256 * t + 4 * lane, K - 4);
        wv[u][t] = *reinterpret_cast<const f32x4*>(w + (size_t)o * K + col);
      }
    }
#pragma unroll
    for (int u = 0; u < CMX_U; ++u) {
      if (i0 + u >= hi) break;
      const int pl = e[u] >> 16;
      if (pl != cur) {
        write_point(cur);
#pragma unroll
        for (int t = 0; t < CMX_T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        cur = pl;
      }
#pragma unroll
      for (int t = 0; t < CMX_T; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[t][q] = fmaf(gv[u], wv[u][t][q], acc[t][q]);
    }
  }
  const bool owner_of_tail = tail_cut && !(cur == lead && lead_cut);
  if (has && !owner_of_tail) write_point(cur);
  __syncthreads();  // carries written
  if (!owner_of_tail) return;
  for (int w2 = wave + 1; w2 < CMX_W && L.carry_pt[w2] == cur; ++w2)
#pragma unroll
    for (int t = 0; t < CMX_T; ++t) {
      const f32x4 cv = *reinterpret_cast<const f32x4*>(&L.carry[w2][256 * t + 4 * lane]);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[t][q] += cv[q];
    }
  write_point(cur);
}

int launch_cmx_bwd(const float* g, const float* gmax, const int32_t* gidx, const float* x,
                   long long ldx, int C, int Npts, int O, int K, const float* w, float* dw,
                   float* db, float* dx, long long lddx, int relu_x, hipStream_t s) {
  PC_REQUIRE(g && gmax && gidx && x && w && C > 0 && Npts > 0 && O > 0 && O <= CMX_MAXO && K > 0 &&
                 O < 65536 && K % 4 == 0 && ldx % 4 == 0 && (!dx || (K <= CMX_MAXK && lddx % 4 == 0)),
             "cmx_bwd: bad shape C=%d N=%d O=%d K=%d", C, Npts, O, K);
  if (dw) {
    hipLaunchKernelGGL(k_cmx_dw, dim3(O, (K + 511) / 512), dim3(128), 0, s, g, gmax, gidx, x, ldx,
                       C, Npts, O, K, dw, db);
    PC_HIP_CHECK_LAUNCH("k_cmx_dw");
  }
  if (dx) {
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_cmx_dx),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(CmxLds)) != hipSuccess) {
        set_error("cmx_bwd: cannot reserve LDS");
        return PCADV_EHIP;
      }
      attr = true;
    }
    hipLaunchKernelGGL(k_cmx_dx, dim3((Npts + CMX_PTS - 1) / CMX_PTS, C), dim3(CMX_W * 64), sizeof(CmxLds),
                       s, g, gmax, gidx, Npts, O, K, w, x, ldx, relu_x, dx, lddx);
    PC_HIP_CHECK_LAUNCH("k_cmx_dx");
  }
  return PCADV_OK;
}

}  // namespace pcadv

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
// point axis into fixed-order slabs (k_gemm_slab_sum).
//
// An optional activation mask multiplies A as it is staged: A[m][k] * [Y > 0]
// with Y stored like A (relu' of the layer output, for dZ = dY relu'(Y)).
#include "common.h"

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
  const float* amask; long long ldm;  // nullable: A *= [amask > 0], stored like A (stride ldm)
  const float* b; long long ldb;
  float* c; long long ldc;
  const float* bias;               // [N] or null
  const float* bias_rows;          // [M / rows_per_group][N] or null
  int rows_per_group;               // bias_rows groups; mode 2: points per cloud
  int M, N, K;
  int relu, accumulate;
  int avec, bvec;                  // 16-B vector loads allowed (aligned base, ld % 4 == 0)
  int ksplit_len;                  // k range per grid.z slab (weight gradients)
  long long slab_stride;           // floats between slabs
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
// l h), f32-level accuracy (the gradients, whose sums cancel heavily)
template <int TA, int TB, int MODE, int NP>
__global__ void __launch_bounds__(GM_T)
k_gemm_x3(GemmP p) {
  constexpr int NPL = NP == 6 ? 3 : 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GemmLds& L = *reinterpret_cast<GemmLds*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = blockIdx.y * GM_BN;
  // mode 2: blockIdx.x = (cloud, row tile of that cloud); rows never straddle clouds
  const int T2 = MODE == 2 ? (p.rows_per_group + GM_BM - 1) / GM_BM : 1;
  const int cl = MODE == 2 ? blockIdx.x / T2 : 0;
  const int m0 = MODE == 2 ? (blockIdx.x % T2) * GM_BM : blockIdx.x * GM_BM;
  const int Mlim = MODE == 2 ? p.rows_per_group : p.M;
  const float* Ab = MODE == 2 ? p.a + (size_t)cl * p.rows_per_group * p.lda : p.a;
  const int kz0 = blockIdx.z * p.ksplit_len;
  const int kz1 = min(p.K, kz0 + p.ksplit_len);
  float* C = p.c + (size_t)blockIdx.z * p.slab_stride;

  // staging: the 128 x 32 f32 tile of A (and of B) is 4096 values, 16 per thread
  f32x4 ra[4], rb[4];
  auto load_tile = [&](int k0) {
    if (TA == 0) {  // A[m][k]: thread = (row tid >> 1, 16 k at 16 (tid & 1))
      const int row = tid >> 1, kk = 16 * (tid & 1);
      const int m = m0 + row;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + kk + 4 * j;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (m < Mlim && k < kz1) {
          const float* src = Ab + (size_t)m * p.lda + k;
          if (p.avec && k + 3 < kz1) {
            v = *reinterpret_cast<const f32x4*>(src);
          } else {
            for (int t = 0; t < 4 && k + t < kz1; ++t) v[t] = src[t];
          }
          if (p.amask) {
            const float* ms = p.amask + (size_t)m * p.ldm + k;
            for (int t = 0; t < 4; ++t)
              if (k + t < kz1 && !(ms[t] > 0.f)) v[t] = 0.f;
          }
        }
        ra[j] = v;
      }
    } else {  // A^T stored: a[k * lda + m]; thread = (k tid >> 3, 16 m at 16 (tid & 7))
      const int kk = tid >> 3, mm = 16 * (tid & 7);
      const int k = k0 + kk;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + mm + 4 * j;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (k < kz1 && m < Mlim) {
          const float* src = Ab + (size_t)k * p.lda + m;
          if (p.avec && m + 3 < Mlim) {
            v = *reinterpret_cast<const f32x4*>(src);
          } else {
            for (int t = 0; t < 4 && m + t < Mlim; ++t) v[t] = src[t];
          }
          if (p.amask) {
            const float* ms = p.amask + (size_t)k * p.ldm + m;
            for (int t = 0; t < 4; ++t)
              if (m + t < Mlim && !(ms[t] > 0.f)) v[t] = 0.f;
          }
        }
        ra[j] = v;
      }
    }
    if (TB == 0) {  // B[n][k]
      const int row = tid >> 1, kk = 16 * (tid & 1);
      const int n = n0 + row;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + kk + 4 * j;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (n < p.N && k < kz1) {
          const float* src = p.b + (size_t)n * p.ldb + k;
          if (p.bvec && k + 3 < kz1) {
            v = *reinterpret_cast<const f32x4*>(src);
          } else {
            for (int t = 0; t < 4 && k + t < kz1; ++t) v[t] = src[t];
          }
        }
        rb[j] = v;
      }
    } else {  // b[k * ldb + n]
      const int kk = tid >> 3, nn = 16 * (tid & 7);
      const int k = k0 + kk;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + nn + 4 * j;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (k < kz1 && n < p.N) {
          const float* src = p.b + (size_t)k * p.ldb + n;
          if (p.bvec && n + 3 < p.N) {
            v = *reinterpret_cast<const f32x4*>(src);
          } else {
            for (int t = 0; t < 4 && n + t < p.N; ++t) v[t] = src[t];
          }
        }
        rb[j] = v;
      }
    }
  };
  auto store_tile = [&]() {
    if (TA == 0) {
      const int row = tid >> 1, kk = 16 * (tid & 1);
      bf16x8g pv[3][2];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        __bf16 o[3];
        split_planes<NPL>(ra[j >> 2][j & 3], o);
#pragma unroll
        for (int q = 0; q < NPL; ++q) pv[q][j >> 3][j & 7] = o[q];
      }
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        *reinterpret_cast<bf16x8g*>(&L.a[q][row * GM_S + kk]) = pv[q][0];
        *reinterpret_cast<bf16x8g*>(&L.a[q][row * GM_S + kk + 8]) = pv[q][1];
      }
    } else {
      const int kk = tid >> 3, mm = 16 * (tid & 7);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        __bf16 o[3];
        split_planes<NPL>(ra[j >> 2][j & 3], o);
#pragma unroll
        for (int q = 0; q < NPL; ++q) L.a[q][(mm + j) * GM_S + kk] = o[q];
      }
    }
    if (TB == 0) {
      const int row = tid >> 1, kk = 16 * (tid & 1);
      bf16x8g pv[3][2];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        __bf16 o[3];
        split_planes<NPL>(rb[j >> 2][j & 3], o);
#pragma unroll
        for (int q = 0; q < NPL; ++q) pv[q][j >> 3][j & 7] = o[q];
      }
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        *reinterpret_cast<bf16x8g*>(&L.b[q][row * GM_S + kk]) = pv[q][0];
        *reinterpret_cast<bf16x8g*>(&L.b[q][row * GM_S + kk + 8]) = pv[q][1];
      }
    } else {
      const int kk = tid >> 3, nn = 16 * (tid & 7);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        __bf16 o[3];
        split_planes<NPL>(rb[j >> 2][j & 3], o);
#pragma unroll
        for (int q = 0; q < NPL; ++q) L.b[q][(nn + j) * GM_S + kk] = o[q];
      }
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  load_tile(kz0);
  for (int k0 = kz0; k0 < kz1; k0 += GM_BK) {
    __syncthreads();  // every wave is done reading the previous tile
    store_tile();
    __syncthreads();
    if (k0 + GM_BK < kz1) load_tile(k0 + GM_BK);  // in flight during the MFMAs
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
      p.part[(size_t)blockIdx.x * p.N + n] = make_int2(b1, b2);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wn + 32 * j + r;
      if (n >= p.N) continue;
      const float bias = p.bias ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + 64 * wm + 32 * i + acc_row(e, lane);
          if (m >= p.M) continue;
          float v = acc[i][j][e] + bias;
          if (p.bias_rows) v += p.bias_rows[(size_t)(m / p.rows_per_group) * p.N + n];
          float* dst = C + (size_t)m * p.ldc + n;
          if (MODE == 1) v += *dst;
          if (p.relu) v = v > 0.f ? v : 0.f;
          *dst = v;
        }
    }
  }
}

// fixed-order sum of nz slabs of M x N (row stride ld) into out (+ column sums)
__global__ void __launch_bounds__(256)
k_gemm_slab_sum(const float* __restrict__ slabs, long long slab_stride, int nz, int M, int N,
                long long ld, float* __restrict__ out, long long ldo, int accumulate) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)M * N) return;
  const int m = (int)(e / N), n = (int)(e % N);
  float s = 0.f;
  for (int z = 0; z < nz; ++z) s += slabs[(size_t)z * slab_stride + (size_t)m * ld + n];
  float* dst = out + (size_t)m * ldo + n;
  *dst = accumulate ? *dst + s : s;
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
// (cloud, channel), re-evaluate the winner (and the runner-up on near-ties) as
// an exact f32 dot product of the input row with the weight row, then apply
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
  const bool near = i2 != 0x7fffffff && !(v1 - v2 > 1e-3f * (fabsf(v1) + fabsf(v2)) + 1e-6f);
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
template <int TA, int TB, int MODE, int NP>
static int gemm_launch(const GemmP& p, int nz, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_x3<TA, TB, MODE, NP>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(GemmLds)) != hipSuccess) {
      set_error("gemm: cannot reserve %zu bytes of LDS", sizeof(GemmLds));
      return PCADV_EHIP;
    }
    attr = true;
  }
  dim3 grid((p.M + GM_BM - 1) / GM_BM, (p.N + GM_BN - 1) / GM_BN, nz);
  hipLaunchKernelGGL((k_gemm_x3<TA, TB, MODE, NP>), grid, dim3(GM_T), sizeof(GemmLds), s, p);
  PC_HIP_CHECK_LAUNCH("k_gemm_x3");
  return PCADV_OK;
}

// C[M][N] (+)= op(A) op(B)^T: see the header comment for ta / tb.
int launch_gemm(const float* a, long long lda, int ta, const float* amask, long long ldm,
                const float* b,
                long long ldb, int tb, float* c, long long ldc, int M, int N, int K,
                const float* bias, const float* bias_rows, int rows_per_group, int relu,
                int accumulate, int precise, hipStream_t s) {
  PC_REQUIRE(a && b && c && M > 0 && N > 0 && K > 0, "gemm: bad shape M=%d N=%d K=%d", M, N, K);
  PC_REQUIRE((ta == 0 && lda >= K) || (ta == 1 && lda >= M), "gemm: bad lda %lld (ta=%d)", lda, ta);
  PC_REQUIRE((tb == 0 && ldb >= K) || (tb == 1 && ldb >= N), "gemm: bad ldb %lld (tb=%d)", ldb, tb);
  PC_REQUIRE(((uintptr_t)a & 3) == 0 && ((uintptr_t)b & 3) == 0 && ((uintptr_t)c & 3) == 0,
             "gemm: operands must be float aligned");
  PC_REQUIRE(ldc >= N, "gemm: bad ldc %lld", ldc);
  PC_REQUIRE(!bias_rows || rows_per_group > 0, "gemm: bias_rows needs rows_per_group");
  PC_REQUIRE(ta == 0 || tb == 1, "gemm: A^T needs B^T (the weight-gradient form)");
  GemmP p{};
  p.a = a; p.lda = lda; p.amask = amask; p.ldm = ldm; p.b = b; p.ldb = ldb; p.c = c; p.ldc = ldc;
  p.bias = bias; p.bias_rows = bias_rows; p.rows_per_group = rows_per_group;
  p.M = M; p.N = N; p.K = K; p.relu = relu; p.accumulate = accumulate;
  p.avec = lda % 4 == 0 && ((uintptr_t)a & 15) == 0;
  p.bvec = ldb % 4 == 0 && ((uintptr_t)b & 15) == 0;
  p.ksplit_len = K;
  if (precise) {
    if (ta == 0 && tb == 0) return accumulate ? gemm_launch<0, 0, 1, 6>(p, 1, s) : gemm_launch<0, 0, 0, 6>(p, 1, s);
    if (ta == 0 && tb == 1) return accumulate ? gemm_launch<0, 1, 1, 6>(p, 1, s) : gemm_launch<0, 1, 0, 6>(p, 1, s);
    return accumulate ? gemm_launch<1, 1, 1, 6>(p, 1, s) : gemm_launch<1, 1, 0, 6>(p, 1, s);
  }
  if (ta == 0 && tb == 0) return accumulate ? gemm_launch<0, 0, 1, 3>(p, 1, s) : gemm_launch<0, 0, 0, 3>(p, 1, s);
  if (ta == 0 && tb == 1) return accumulate ? gemm_launch<0, 1, 1, 3>(p, 1, s) : gemm_launch<0, 1, 0, 3>(p, 1, s);
  return accumulate ? gemm_launch<1, 1, 1, 3>(p, 1, s) : gemm_launch<1, 1, 0, 3>(p, 1, s);
}

// weight gradient dW[N][K'] (+)= sum over M' points of dZ[m][n] X[m][k]:
// A = dZ^T (stored [M'][N], row stride ldz), B = X^T (stored [M'][K'], ldx),
// the point axis split into nz fixed-order slabs in the workspace.
size_t gemm_wgrad_workspace_bytes(int rows, int O, int Kin) {
  const int nz = rows >= 4096 ? min(32, rows / 1024) : 1;
  return (size_t)nz * O * Kin * sizeof(float) + 256;
}

int launch_gemm_wgrad(const float* dz, long long ldz, const float* ymask, long long ldm,
                      const float* x, long long ldx, int rows, int O, int Kin, float* dw,
                      long long ldo, int accumulate, void* ws, size_t ws_bytes, hipStream_t s) {
  PC_REQUIRE(dz && x && dw && rows > 0 && O > 0 && Kin > 0 && ldo >= Kin, "gemm_wgrad: bad shape");

  const int nz = rows >= 4096 ? min(32, rows / 1024) : 1;
  PC_REQUIRE(ws && ws_bytes >= gemm_wgrad_workspace_bytes(rows, O, Kin), "gemm_wgrad: workspace");
  GemmP p{};
  p.a = dz; p.lda = ldz; p.amask = ymask; p.ldm = ldm; p.b = x; p.ldb = ldx;
  p.c = static_cast<float*>(ws); p.ldc = Kin;
  p.M = O; p.N = Kin; p.K = rows;
  p.avec = ldz % 4 == 0 && ((uintptr_t)dz & 15) == 0;
  p.bvec = ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
  p.ksplit_len = ((rows + nz - 1) / nz + GM_BK - 1) / GM_BK * GM_BK;
  p.slab_stride = (long long)O * Kin;
  PC_TRY_GEMM((gemm_launch<1, 1, 0, 6>(p, nz, s)));
  const long long tot = (long long)O * Kin;
  hipLaunchKernelGGL(k_gemm_slab_sum, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     static_cast<const float*>(ws), p.slab_stride, nz, O, Kin, (long long)Kin, dw,
                     ldo, accumulate);
  PC_HIP_CHECK_LAUNCH("k_gemm_slab_sum");
  return PCADV_OK;
}

size_t colsum_workspace_bytes(int M, int N) {
  const int nchunk = (M + 1023) / 1024;
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
  const int nchunk = (M + 1023) / 1024;
  PC_REQUIRE(ws && ws_bytes >= colsum_workspace_bytes(M, N), "colsum: workspace");
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(k_colsum_part, dim3((N + 63) / 64, nchunk), dim3(256), 0, s, x, ymask, ld,
                     ldm, M, N, 1024, part);
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
                       size_t ws_bytes, hipStream_t s) {
  PC_REQUIRE(x && w && gmax && gidx && C > 0 && Npts > 0 && K > 0 && O > 0,
             "conv_max_x3: bad shape");
  PC_REQUIRE(K % 32 == 0 && ldx % 4 == 0, "conv_max_x3: K %% 32 and ldx %% 4 required");
  PC_REQUIRE(ws && ws_bytes >= conv_max_x3_workspace_bytes(C, Npts, O), "conv_max_x3: workspace");
  const int T = (Npts + GM_BM - 1) / GM_BM;
  int2* part = static_cast<int2*>(ws);
  {
    GemmP p{};
    p.a = x; p.lda = ldx; p.b = w; p.ldb = K;
    p.c = gmax; p.ldc = O;
    p.avec = ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
    p.bvec = K % 4 == 0 && ((uintptr_t)w & 15) == 0;
    p.rows_per_group = Npts;
    p.M = C * Npts; p.N = O; p.K = K; p.ksplit_len = K;
    p.part = part;
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_gemm_x3<0, 0, 2, 3>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(GemmLds)) != hipSuccess) {
        set_error("conv_max_x3: cannot reserve LDS");
        return PCADV_EHIP;
      }
      attr = true;
    }
    hipLaunchKernelGGL((k_gemm_x3<0, 0, 2, 3>), dim3(C * T, (O + GM_BN - 1) / GM_BN, 1), dim3(GM_T),
                       sizeof(GemmLds), s, p);
    PC_HIP_CHECK_LAUNCH("k_gemm_x3 (max)");
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
  const int nb = (M + 255) / 256;
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(k_row_ce, dim3(nb), dim3(256), 0, s, logits, ld, labels, M, Ccls, scale,
                     dlogits, part);
  PC_HIP_CHECK_LAUNCH("k_row_ce");
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
  for (int c = 0; c < C; ++c) {
    const float gv = gmax[(size_t)c * O + o] > 0.f ? g[(size_t)c * O + o] : 0.f;
    sb += gv;
    if (gv == 0.f || k >= K) continue;
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + (size_t)(c * Npts + gidx[(size_t)c * O + o]) * ldx + k);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = fmaf(gv, v[t], acc[t]);
  }
  if (k < K) *reinterpret_cast<f32x4*>(dw + (size_t)o * K + k) = acc;
  if (blockIdx.y == 0 && threadIdx.x == 0 && db) db[o] = sb;
}

// One workgroup per (cloud, 256-column block of K).  The cloud's live hits
// (g' != 0) are bucketed by argmax point (counting sort in LDS), each bucket is
// ordered by o, and each thread then walks the hits for its column, adding one
// sum per point: a fixed summation order, bitwise reproducible.
constexpr int CMX_MAXO = 4096, CMX_MAXP = 4096;
struct CmxLds {
  int cnt[CMX_MAXP];   // hits per point, then bucket starts
  int fill[CMX_MAXP];
  int ho[CMX_MAXO];    // o of each hit, bucketed by point
  int hp[CMX_MAXO];    // point of each hit
  int part[256];
  int n;
};

__global__ void __launch_bounds__(256)
k_cmx_dx(const float* __restrict__ g, const float* __restrict__ gmax,
         const int32_t* __restrict__ gidx, int Npts, int O, int K, const float* __restrict__ w,
         float* __restrict__ dx, long long lddx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  CmxLds& L = *reinterpret_cast<CmxLds*>(smem);
  const int c = blockIdx.x, tid = threadIdx.x, col = blockIdx.y * 256 + tid;
  for (int p = tid; p < Npts; p += 256) {
    L.cnt[p] = 0;
    L.fill[p] = 0;
  }
  __syncthreads();
  for (int o = tid; o < O; o += 256)
    if (gmax[(size_t)c * O + o] > 0.f && g[(size_t)c * O + o] != 0.f)
      atomicAdd(&L.cnt[gidx[(size_t)c * O + o]], 1);
  __syncthreads();
  // exclusive scan of cnt over the points: per-thread runs, then the run totals
  const int per = (Npts + 255) / 256, p0 = tid * per;
  int run = 0;
  for (int p = p0; p < min(Npts, p0 + per); ++p) run += L.cnt[p];
  L.part[tid] = run;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int t = 0; t < 256; ++t) {
      const int v = L.part[t];
      L.part[t] = acc;
      acc += v;
    }
    L.n = acc;
  }
  __syncthreads();
  int off = L.part[tid];
  for (int p = p0; p < min(Npts, p0 + per); ++p) {
    const int v = L.cnt[p];
    L.cnt[p] = off;
    off += v;
  }
  __syncthreads();
  for (int o = tid; o < O; o += 256)
    if (gmax[(size_t)c * O + o] > 0.f && g[(size_t)c * O + o] != 0.f) {
      const int p = gidx[(size_t)c * O + o];
      const int pos = L.cnt[p] + atomicAdd(&L.fill[p], 1);
      L.ho[pos] = o;
      L.hp[pos] = p;
    }
  __syncthreads();
  // order each bucket by o (buckets are short: insertion sort, a thread per point)
  for (int p = tid; p < Npts; p += 256) {
    const int s0 = L.cnt[p], len = L.fill[p];
    for (int i = s0 + 1; i < s0 + len; ++i) {
      const int v = L.ho[i];
      int j = i - 1;
      while (j >= s0 && L.ho[j] > v) {
        L.ho[j + 1] = L.ho[j];
        --j;
      }
      L.ho[j + 1] = v;
    }
  }
  __syncthreads();
  if (col >= K) return;
  const int n = L.n;
  float acc = 0.f;
  int cur = n > 0 ? L.hp[0] : -1;
  for (int i = 0; i < n; ++i) {
    const int p = L.hp[i], o = L.ho[i];
    if (p != cur) {
      float* d = dx + (size_t)(c * Npts + cur) * lddx + col;
      *d += acc;
      acc = 0.f;
      cur = p;
    }
    acc = fmaf(g[(size_t)c * O + o], w[(size_t)o * K + col], acc);
  }
  if (n > 0) {
    float* d = dx + (size_t)(c * Npts + cur) * lddx + col;
    *d += acc;
  }
}

int launch_cmx_bwd(const float* g, const float* gmax, const int32_t* gidx, const float* x,
                   long long ldx, int C, int Npts, int O, int K, const float* w, float* dw,
                   float* db, float* dx, long long lddx, hipStream_t s) {
  PC_REQUIRE(g && gmax && gidx && x && w && C > 0 && Npts > 0 && Npts <= CMX_MAXP && O > 0 &&
                 O <= CMX_MAXO && K > 0 && K % 4 == 0 && ldx % 4 == 0,
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
    hipLaunchKernelGGL(k_cmx_dx, dim3(C, (K + 255) / 256), dim3(256), sizeof(CmxLds), s, g, gmax,
                       gidx, Npts, O, K, w, dx, lddx);
    PC_HIP_CHECK_LAUNCH("k_cmx_dx");
  }
  return PCADV_OK;
}

}  // namespace pcadv

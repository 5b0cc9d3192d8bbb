// Small dense layers of the hot path on gfx950: the PointNetCls head
// (models/pointnet.py:191-202: fc1+ReLU, fc2+Dropout+ReLU, fc3) and the
// DeepConvDiscNet MLP (models/discriminator.py:33-51: five 1x1 convs on
// B x C x 1 with LeakyReLU(0.2), then Linear(64, 1)).
//
// M (clouds / D rows) is 64..96, so every layer is a few MFLOP and the cost is
// latency, not arithmetic.  Each 16x16 output tile runs on v_mfma_f32_16x16x4_f32
// (exact f32); the reduction dimension is split over up to 16 waves of one
// block, every wave issues ALL of its operand loads before its first MFMA, and
// the partial tiles meet once in LDS in a fixed order (deterministic).  The
// weight-gradient job (reduction over the <= 128 rows) gives each wave its own
// tile instead.  Dropout masks and activation derivatives are applied where
// the operands are loaded.
#include "common.h"

namespace pcadv {

struct DropSpec {
  const float* mask;    // [M][N] {0,1} or nullptr
  const int32_t* step;  // device step counter for the Philox draw, or nullptr
  uint64_t seed;
  float p;
};

__device__ __forceinline__ bool has_drop(const DropSpec& d) { return d.mask || d.step; }

__device__ __forceinline__ float drop_scale(const DropSpec& d, int m, int n, int N) {
  if (d.mask) return d.mask[(size_t)m * N + n] * (1.0f / (1.0f - d.p));
  if (d.step) {
    const float u = rng_uniform(d.seed, (uint32_t)*d.step, RNG_DROPOUT, (uint32_t)(m * N + n));
    return u >= d.p ? 1.0f / (1.0f - d.p) : 0.f;
  }
  return 1.f;
}

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// dz = dy * act'(y) * s at (m, n)
__device__ __forceinline__ float dz_at(const float* __restrict__ dy, const float* __restrict__ y,
                                       int act, const DropSpec& drop, int m, int n, int N) {
  float g = dy[(size_t)m * N + n];
  if (act != ACT_NONE) g *= act_bwd(y[(size_t)m * N + n], act);
  if (has_drop(drop)) g *= drop_scale(drop, m, n, N);
  return g;
}

enum Op { OP_FWD = 0, OP_BWD_DATA = 1, OP_BWD_WEIGHT = 2 };

struct GemmArgs {
  // forward: y = act(s * (x w^T + b)); backward: dy/y/act/drop define dz
  const float* x;
  const float* w;
  const float* b;
  float* y;  // forward output
  const float* dy;
  const float* yact;
  int act;
  DropSpec drop;
  float* dx;
  float* dw;
  float* db;
  int M, N, K, m_w;
};

constexpr int MAXC = 8;  // 16-deep k chunks per wave (reduction <= 128 per wave)
constexpr int SPLITC = 4;  // split jobs: <= 64 per wave (16 waves cover 1024)

// Load the (k = kk..kk+3) A and B operand values of lane (r) for output tile
// (r0, c0): A row r0 + r, B column c0 + r.
template <int OP>
__device__ __forceinline__ void load_ab(const GemmArgs& g, int r0, int c0, int r, int kk,
                                        float* a, float* b) {
  if (OP == OP_FWD) {
    // out[m][n] = sum_k x[m][k] w[n][k]
    const int m = r0 + r, n = c0 + r;
    const f32x4v z = {0.f, 0.f, 0.f, 0.f};
    f32x4v av = (m < g.M && kk < g.K) ? *reinterpret_cast<const f32x4v*>(g.x + (size_t)m * g.K + kk) : z;
    f32x4v bv = (n < g.N && kk < g.K) ? *reinterpret_cast<const f32x4v*>(g.w + (size_t)n * g.K + kk) : z;
    a[0] = av.x; a[1] = av.y; a[2] = av.z; a[3] = av.w;
    b[0] = bv.x; b[1] = bv.y; b[2] = bv.z; b[3] = bv.w;
  } else if (OP == OP_BWD_DATA) {
    // dx[m][k] = sum_n dz[m][n] w[n][k]
    const int m = r0 + r, k = c0 + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = kk + j;
      a[j] = (m < g.M && n < g.N) ? dz_at(g.dy, g.yact, g.act, g.drop, m, n, g.N) : 0.f;
      b[j] = (n < g.N && k < g.K) ? g.w[(size_t)n * g.K + k] : 0.f;
    }
  } else {
    // dw[n][k] = sum_{m < m_w} dz[m][n] x[m][k]
    const int n = r0 + r, k = c0 + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = kk + j;
      a[j] = (m < g.m_w && n < g.N) ? dz_at(g.dy, g.yact, g.act, g.drop, m, n, g.N) : 0.f;
      b[j] = (m < g.m_w && k < g.K) ? g.x[(size_t)m * g.K + k] : 0.f;
    }
  }
}

// One wave: 16x16 tile (r0, c0) over reduction [k0, k1) with nch <= MAXC chunks.
template <int OP, int NC>
__device__ __forceinline__ f32x4v wave_tile(const GemmArgs& g, int r0, int c0, int k0, int nch,
                                            int lane, float* asum) {
  const int r = lane & 15, q = lane >> 4;
  float a[NC][4], b[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c < nch) {
      load_ab<OP>(g, r0, c0, r, k0 + 16 * c + 4 * q, a[c], b[c]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) a[c][j] = b[c][j] = 0.f;
    }
  }
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c < nch) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc = mfma16(a[c][j], b[c][j], acc);
        s += a[c][j];
      }
    }
  }
  *asum = s;
  return acc;
}

// Split-reduction job (forward, backward-data): block = one 16x16 tile, wave w
// takes reduction slice w.  Tiles are numbered row-major over (rows, cols).
template <int OP>
__device__ void split_job(const GemmArgs& g, int tile, int rows, int cols, int R, int S, int L,
                          float* red) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ctiles = (cols + 15) / 16;
  const int r0 = (tile / ctiles) * 16, c0 = (tile % ctiles) * 16;
  const int k0 = wave * L;
  int nch = 0;
  if (k0 < R) nch = min(L, R - k0 + 15) / 16;
  float s;
  f32x4v acc = wave_tile<OP, SPLITC>(g, r0, c0, k0, nch, lane, &s);
  const int col = lane & 15, q = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) red[wave * 256 + (4 * q + j) * 16 + col] = acc[j];
  __syncthreads();
  for (int e = tid; e < 256; e += blockDim.x) {
    const int row = e >> 4, cc = e & 15;
    float v = 0.f;
    for (int w = 0; w < S; ++w) v += red[w * 256 + e];
    const int m = r0 + row, n = c0 + cc;
    if (m < rows && n < cols) {
      if (OP == OP_FWD) {
        v += g.b[n];
        if (has_drop(g.drop)) v *= drop_scale(g.drop, m, n, g.N);
        g.y[(size_t)m * g.N + n] = act_fwd(v, g.act);
      } else {
        g.dx[(size_t)m * g.K + n] = v;
      }
    }
  }
}

// Weight-gradient job: every wave owns one 16x16 tile of dw (rows n, cols k)
// and the full reduction over the m_w rows; k-tile 0 also produces db.
__device__ void weight_job(const GemmArgs& g, int tile, int ntiles_total) {
  const int lane = threadIdx.x & 63;
  if (tile >= ntiles_total) return;
  const int ctiles = (g.K + 15) / 16;
  const int r0 = (tile / ctiles) * 16, c0 = (tile % ctiles) * 16;
  const int nch = (g.m_w + 15) / 16;
  float s;
  f32x4v acc = wave_tile<OP_BWD_WEIGHT, MAXC>(g, r0, c0, 0, nch, lane, &s);
  const int col = lane & 15, q = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = r0 + 4 * q + j, k = c0 + col;
    if (n < g.N && k < g.K) g.dw[(size_t)n * g.K + k] = acc[j];
  }
  if (g.db && c0 == 0) {
    // lane (r, q) summed dz[m][r0 + r] over its m's; add the 4 q groups
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (q == 0 && r0 + col < g.N) g.db[r0 + col] = s;
  }
}

__global__ void __launch_bounds__(1024)
k_linear_fwd(GemmArgs g, int S, int L) {
  __shared__ float red[16 * 256];
  split_job<OP_FWD>(g, blockIdx.x, g.M, g.N, g.K, S, L, red);
}

// blocks [0, nbx): dx tiles (split over S waves); the rest: dw tiles, S per block
__global__ void __launch_bounds__(1024)
k_linear_bwd(GemmArgs g, int S, int L, int nbx, int nwt) {
  __shared__ float red[16 * 256];
  if ((int)blockIdx.x < nbx) {
    split_job<OP_BWD_DATA>(g, blockIdx.x, g.M, g.K, g.N, S, L, red);
  } else {
    weight_job(g, (blockIdx.x - nbx) * S + (threadIdx.x >> 6), nwt);
  }
}

static void split_cfg(int R, int* S, int* L) {
  int s = (R + 63) / 64;
  if (s < 1) s = 1;
  if (s > 16) s = 16;
  int l = ((R + s - 1) / s + 15) / 16 * 16;
  *S = s;
  *L = l;
}

int launch_linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int N,
                      int K, int act, const float* mask, const int32_t* step, uint64_t seed,
                      float p, hipStream_t s) {
  PC_REQUIRE(M > 0 && N > 0 && K > 0 && K % 4 == 0 && K <= 16 * 16 * SPLITC,
             "linear_fwd: bad shape M=%d N=%d K=%d", M, N, K);
  GemmArgs g{};
  g.x = x; g.w = w; g.b = b; g.y = y; g.act = act;
  g.drop = DropSpec{mask, step, seed, p};
  g.M = M; g.N = N; g.K = K;
  int S, L;
  split_cfg(K, &S, &L);
  const int tiles = ((M + 15) / 16) * ((N + 15) / 16);
  hipLaunchKernelGGL(k_linear_fwd, dim3(tiles), dim3(64 * S), 0, s, g, S, L);
  PC_HIP_CHECK_LAUNCH("k_linear_fwd");
  return PCADV_OK;
}

int launch_linear_bwd(const float* dy, const float* y, int act, const float* mask,
                      const int32_t* step, uint64_t seed, float p, const float* x, const float* w,
                      float* dx, float* dw, float* db, int M, int m_w, int N, int K,
                      hipStream_t s) {
  PC_REQUIRE(M > 0 && N > 0 && K > 0 && K % 4 == 0 && m_w >= 0 && m_w <= M &&
                 m_w <= 16 * MAXC && N <= 16 * 16 * SPLITC,
             "linear_bwd: bad shape M=%d m_w=%d N=%d K=%d", M, m_w, N, K);
  GemmArgs g{};
  g.x = x; g.w = w; g.dy = dy; g.yact = y; g.act = act;
  g.drop = DropSpec{mask, step, seed, p};
  g.dx = dx; g.dw = dw; g.db = db;
  g.M = M; g.N = N; g.K = K; g.m_w = m_w;
  int S, L;
  split_cfg(N, &S, &L);
  const int nbx = dx ? ((M + 15) / 16) * ((K + 15) / 16) : 0;
  const int nwt = dw ? ((N + 15) / 16) * ((K + 15) / 16) : 0;
  const int nbw = (nwt + S - 1) / S;
  if (nbx + nbw == 0) return PCADV_OK;
  hipLaunchKernelGGL(k_linear_bwd, dim3(nbx + nbw), dim3(64 * S), 0, s, g, S, L, nbx, nwt);
  PC_HIP_CHECK_LAUNCH("k_linear_bwd");
  return PCADV_OK;
}

}  // namespace pcadv

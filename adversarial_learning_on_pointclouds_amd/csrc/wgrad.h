// Weight gradients of the small dense layers (fc1..fc3 of PointNetCls, the
// discriminator's 1x1 convs) in the linear-backward launches (linear.hip): a
// wave form (one 16x16 tile per wave, operands loaded straight to registers)
// and a block form (operands staged in LDS), bitwise the same results.
//
//   dw[n][k] = sum_{m < m_w} dz[m][n] x[m][k],  db[n] = sum_{m < m_w} dz[m][n]
//
// dz is stored as is (its producer applied the activation derivative and the
// dropout mask).  One 16x16 tile of dw per wave on v_mfma_f32_16x16x4_f32
// (exact f32), the reduction over the rows in a fixed order: row m enters MFMA
// step 4 (m / 16) + m % 4 of the tile's single accumulation chain, lane group
// (m % 16) / 4; any number of rows (slabs of 16 WG_MAXC rows).
#pragma once
#include "common.h"

namespace pcadv {

struct WgradJob {
  const float* dz;  // [M][N] (rows >= m_w are not read)
  const float* x;   // [M][K]
  float* dw;        // [N][K]
  float* db;        // [N] or nullptr
  int N, K, m_w;
  int tiles;        // launch bookkeeping (linear.hip)
};

constexpr int WG_MAXC = 8;  // 16-row chunks per slab (128 rows)

typedef float wg_f32x4 __attribute__((ext_vector_type(4)));

// One wave: the (r0, c0) tile over rows [m0, m0 + 16 nch), NC >= nch chunks,
// accumulated onto acc / *asum; chunks past nch load clamped addresses and
// contribute zeros, so every load is issued before the first MFMA.
template <int NC>
__device__ __forceinline__ wg_f32x4 wgrad_tile(const WgradJob& j, int r0, int c0, int m0, int nch,
                                               int lane, float* asum, wg_f32x4 acc) {
  const int r = lane & 15, q = lane >> 4;
  const int n = r0 + r, k = c0 + r;
  float a[NC][4], b[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int m = m0 + 16 * c + 4 * q + jj;
      const bool va = c < nch && m < j.m_w && n < j.N;
      const float dv = j.dz[(size_t)(va ? m : 0) * j.N + (va ? n : 0)];
      a[c][jj] = va ? dv : 0.f;
      const bool vb = c < nch && m < j.m_w && k < j.K;
      const float xv = j.x[(size_t)(vb ? m : 0) * j.K + (vb ? k : 0)];
      b[c][jj] = vb ? xv : 0.f;
    }
  }
  float s = *asum;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c][jj], b[c][jj], acc, 0, 0, 0);
      s += a[c][jj];
    }
  }
  *asum = s;
  return acc;
}

// the tile's outputs: dw rows r0 + 4 q + jj, column c0 + (lane & 15); db from
// the lane sums of the 4 lane groups
__device__ __forceinline__ void wgrad_store(const WgradJob& j, int r0, int c0, wg_f32x4 acc,
                                            float s, int lane) {
  const int col = lane & 15, q = lane >> 4;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int n = r0 + 4 * q + jj, k = c0 + col;
    if (n < j.N && k < j.K) j.dw[(size_t)n * j.K + k] = acc[jj];
  }
  if (j.db && c0 == 0) {
    // lane (r, q) summed dz[m][r0 + r] over its m's; add the 4 q groups
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (q == 0 && r0 + col < j.N) j.db[r0 + col] = s;
  }
}

// Tile `tile` of job j on this wave (all 64 lanes take part).
__device__ __forceinline__ void wgrad_wave(const WgradJob& j, int tile, int lane) {
  const int ctiles = (j.K + 15) / 16;
  const int r0 = (tile / ctiles) * 16, c0 = (tile % ctiles) * 16;
  float s = 0.f;
  wg_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int m0 = 0; m0 < j.m_w; m0 += 16 * WG_MAXC) {
    const int nch = min(WG_MAXC, (j.m_w - m0 + 15) / 16);
    // the load count follows the chunk count (m_w <= 64 at B = 32: half the loads)
    acc = nch <= WG_MAXC / 2 ? wgrad_tile<WG_MAXC / 2>(j, r0, c0, m0, nch, lane, &s, acc)
                             : wgrad_tile<WG_MAXC>(j, r0, c0, m0, nch, lane, &s, acc);
  }
  wgrad_store(j, r0, c0, acc, s, lane);
}

// Block-level form (a block of `nwaves` waves; what the backward launches
// use): region `region` of dw = rows [n0, n0 + 64) x columns [k0, k0 + 32),
// its eight tiles spread over the waves.  Per slab of 16 WG_MAXC rows the
// block stages dz[m][n0:n0 + 64] and x[m][k0:k0 + 32] in LDS with 16-byte
// loads (a vector-memory instruction per KiB instead of per 256 B: the wave
// form's column walks make a launch issue-bound), then reads the fragments
// from there.  Same operands and MFMA order as wgrad_wave: bitwise the same dw
// and db.  Needs N % 4 == 0, K % 4 == 0 and nwaves >= WGB_MIN_WAVES; LDS:
// WGB_LDS_FLOATS.
constexpr int WGB_N = 64, WGB_K = 32;
constexpr int WGB_ZS = WGB_N + 4, WGB_XS = WGB_K + 4;  // 4q rows apart -> 16q banks apart
constexpr int WGB_LDS_FLOATS = 16 * WG_MAXC * (WGB_ZS + WGB_XS);
constexpr int WGB_MIN_WAVES = 4;
constexpr int WGB_TILES = (WGB_N / 16) * (WGB_K / 16);

__host__ __device__ inline int wgrad_regions(int N, int K) {
  return ((N + WGB_N - 1) / WGB_N) * ((K + WGB_K - 1) / WGB_K);
}

__device__ __forceinline__ void wgrad_region(const WgradJob& j, int region, float* lds, int nwaves) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nthr = 64 * nwaves;
  const int kreg = (j.K + WGB_K - 1) / WGB_K;
  const int n0 = (region / kreg) * WGB_N, k0 = (region % kreg) * WGB_K;
  float* zl = lds;
  float* xl = lds + 16 * WG_MAXC * WGB_ZS;
  constexpr int TPW = WGB_TILES / WGB_MIN_WAVES;  // tiles per wave at most
  wg_f32x4 acc[TPW];
  float s[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    acc[i] = wg_f32x4{0.f, 0.f, 0.f, 0.f};
    s[i] = 0.f;
  }
  const int r = lane & 15, q = lane >> 4;
  for (int m0 = 0; m0 < j.m_w; m0 += 16 * WG_MAXC) {
    const int nch = min(WG_MAXC, (j.m_w - m0 + 15) / 16), rows = 16 * nch;
    if (m0 > 0) __syncthreads();  // the previous slab's fragments are read
    // all the 16-byte loads of a thread are in flight before its first LDS
    // store; pieces past the staged rows issue no load
    constexpr int PZ = 16 * WG_MAXC * (WGB_N / 4) / (64 * WGB_MIN_WAVES);
    constexpr int PX = 16 * WG_MAXC * (WGB_K / 4) / (64 * WGB_MIN_WAVES);
    wg_f32x4 vz[PZ], vx[PX];
#pragma unroll
    for (int u = 0; u < PZ; ++u) {
      const int e = tid + u * nthr, m = e >> 4, n = n0 + 4 * (e & 15);
      vz[u] = wg_f32x4{0.f, 0.f, 0.f, 0.f};
      if (m < rows && m0 + m < j.m_w && n < j.N)
        vz[u] = *reinterpret_cast<const wg_f32x4*>(j.dz + (size_t)(m0 + m) * j.N + n);
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int e = tid + u * nthr, m = e >> 3, k = k0 + 4 * (e & 7);
      vx[u] = wg_f32x4{0.f, 0.f, 0.f, 0.f};
      if (m < rows && m0 + m < j.m_w && k < j.K)
        vx[u] = *reinterpret_cast<const wg_f32x4*>(j.x + (size_t)(m0 + m) * j.K + k);
    }
#pragma unroll
    for (int u = 0; u < PZ; ++u) {
      const int e = tid + u * nthr, m = e >> 4;
      if (m < rows) *reinterpret_cast<wg_f32x4*>(zl + m * WGB_ZS + 4 * (e & 15)) = vz[u];
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int e = tid + u * nthr, m = e >> 3;
      if (m < rows) *reinterpret_cast<wg_f32x4*>(xl + m * WGB_XS + 4 * (e & 7)) = vx[u];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = wave + i * nwaves;
      if (t >= WGB_TILES) break;
      const int nt = t / (WGB_K / 16), kt = t % (WGB_K / 16);
      for (int c = 0; c < nch; ++c) {
        float a[4], b[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int m = 16 * c + 4 * q + jj;
          a[jj] = zl[m * WGB_ZS + 16 * nt + r];
          b[jj] = xl[m * WGB_XS + 16 * kt + r];
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[jj], b[jj], acc[i], 0, 0, 0);
          s[i] += a[jj];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + i * nwaves;
    if (t >= WGB_TILES) break;
    const int nt = t / (WGB_K / 16), kt = t % (WGB_K / 16);
    const int r0 = n0 + 16 * nt, c0 = k0 + 16 * kt;
    if (r0 < j.N && c0 < j.K) wgrad_store(j, r0, c0, acc[i], s[i], lane);
  }
}

}  // namespace pcadv

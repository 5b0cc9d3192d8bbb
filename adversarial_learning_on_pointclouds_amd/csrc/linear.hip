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
#include "wgrad.h"

namespace pcadv {

struct DropSpec {
  const float* mask;    // [M][N] {0,1} or nullptr
  const int32_t* step;  // device step counter for the Philox draw, or nullptr
  uint64_t seed;
  float p;
  // Philox row of output row m: m + (m < split ? off_lo : off_hi), so a rank of
  // a data-parallel step draws the rows of the global batch it holds (the GT
  // rows [0, split) and the no-GT rows after them shift separately); all 0 =
  // the launch's own rows
  int split, off_lo, off_hi;
};

// dropout source, fixed per launch (a template parameter: the operand loads
// below are then straight-line code the compiler can issue back to back)
enum DropMode { DM_NONE = 0, DM_MASK = 1, DM_RNG = 2 };

static int drop_mode(const DropSpec& d) { return d.mask ? DM_MASK : (d.step ? DM_RNG : DM_NONE); }

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
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
  int diag;  // forward: add the k x k identity to the flattened output (0: off)
  float* mask_out;  // forward, device-drawn dropout: store the {0,1} mask here
  // backward-data output mask: dx *= act'(x) (* ox_mask * ox_keep), i.e. dx is
  // stored as the layer below's dz, so its backward reads one operand as is
  int ox_act;
  const float* ox_mask;
  float ox_keep;
  int stamp_slot;  // diagnostic build: row of g_lin_stamps (-1: none)
  // backward data: chained tile product (LinBwdExtra.chain_*), chain_n <= 48
  const float* chain_w;
  float* chain_out;
  int chain_row0, chain_n;
};

#ifdef PCADV_STAMPS
// diagnostic build only: wave 0's timestamps per block (s_memrealtime):
// [launch][block][start, tile summed, partials met, end, operands landed, loads issued]
__device__ uint64_t g_lin_stamps[16][256][6];
#define LSTAMP(g, k)                                                            \
  do {                                                                          \
    if (threadIdx.x == 0 && (g).stamp_slot >= 0 && blockIdx.x < 256)            \
      g_lin_stamps[(g).stamp_slot][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
static int g_lin_seq = 0;
static int next_stamp_slot() { return g_lin_seq < 16 ? g_lin_seq++ : -1; }
int lin_stamps_read(uint64_t* host, int reset) {
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lin_stamps), sizeof(g_lin_stamps)) != hipSuccess)
    return PCADV_EHIP;
  if (reset) g_lin_seq = 0;
  return PCADV_OK;
}
#else
#define LSTAMP(g, k) do { } while (0)
static int next_stamp_slot() { return -1; }
#endif

// dropout scale s at (m, n) of an [M][N] output
template <int DM>
__device__ __forceinline__ float drop_scale(const GemmArgs& g, size_t i, int m, int n,
                                            uint32_t step) {
  const float keep = 1.0f / (1.0f - g.drop.p);
  if (DM == DM_MASK) return g.drop.mask[i] * keep;
  if (DM == DM_RNG)
  {
    const int gm = m + (m < g.drop.split ? g.drop.off_lo : g.drop.off_hi);
    return rng_uniform(g.drop.seed, step, RNG_DROPOUT, (uint32_t)(gm * g.N + n)) >= g.drop.p ? keep
                                                                                             : 0.f;
  }
  return 1.f;
}

// dz = dy * act'(y) * s at (m, n), 0 outside; the loads are unconditional
// (clamped address) so a wave issues all of them before the first use
template <int ACT, int DM>
__device__ __forceinline__ float dz_at(const GemmArgs& g, int m, int n, bool valid,
                                       uint32_t step) {
  const size_t i = (size_t)(valid ? m : 0) * g.N + (valid ? n : 0);
  float v = g.dy[i];
  if (ACT != ACT_NONE) v *= act_bwd(g.yact[i], ACT);
  if (DM != DM_NONE) v *= drop_scale<DM>(g, i, m, n, step);
  return valid ? v : 0.f;
}

constexpr int MAXC = 8;  // 16-deep k chunks per wave (reduction <= 128 per wave)
constexpr int SPLITC = 4;  // split jobs: <= 64 per wave (16 waves cover 1024)

// Load the (k = kk..kk+3) A and B operand values of lane (r) for output tile
// (r0, c0): A row r0 + r, B column c0 + r.
template <int OP, int ACT, int DM>
__device__ __forceinline__ void load_ab(const GemmArgs& g, int r0, int c0, int r, int kk, bool cv,
                                        uint32_t step, float* a, float* b) {
  if (OP == OP_FWD) {
    // out[m][n] = sum_k x[m][k] w[n][k]  (K % 4 == 0: kk < K covers all four)
    const int m = r0 + r, n = c0 + r;
    const bool va = cv && m < g.M && kk < g.K, vb = cv && n < g.N && kk < g.K;
    const f32x4v av = *reinterpret_cast<const f32x4v*>(
        g.x + (size_t)(va ? m : 0) * g.K + (va ? kk : 0));
    const f32x4v bv = *reinterpret_cast<const f32x4v*>(
        g.w + (size_t)(vb ? n : 0) * g.K + (vb ? kk : 0));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = va ? av[j] : 0.f;
      b[j] = vb ? bv[j] : 0.f;
    }
  } else if (OP == OP_BWD_DATA) {
    // dx[m][k] = sum_n dz[m][n] w[n][k]
    const int m = r0 + r, k = c0 + r;
    if (ACT == ACT_NONE && DM == DM_NONE && (g.N & 3) == 0) {
      // dz stored as is (the producer applied the masks): one 16-B load
      const bool va = cv && m < g.M && kk < g.N;
      const f32x4v av = *reinterpret_cast<const f32x4v*>(
          g.dy + (size_t)(va ? m : 0) * g.N + (va ? kk : 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = va ? av[j] : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        a[j] = dz_at<ACT, DM>(g, m, kk + j, cv && m < g.M && kk + j < g.N, step);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = kk + j;
      const bool vb = cv && n < g.N && k < g.K;
      const float wv = g.w[(size_t)(vb ? n : 0) * g.K + (vb ? k : 0)];
      b[j] = vb ? wv : 0.f;
    }
  } else {
    // dw[n][k] = sum_{m < m_w} dz[m][n] x[m][k]
    const int n = r0 + r, k = c0 + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = kk + j;
      a[j] = dz_at<ACT, DM>(g, m, n, cv && m < g.m_w && n < g.N, step);
      const bool vb = cv && m < g.m_w && k < g.K;
      const float xv = g.x[(size_t)(vb ? m : 0) * g.K + (vb ? k : 0)];
      b[j] = vb ? xv : 0.f;
    }
  }
}

// One wave: 16x16 tile (r0, c0) over reduction [k0, k0 + 16*nch), nch <= NC.
// Chunks past nch load clamped addresses and contribute zeros, so the loop is
// branch-free and every load is issued before the first MFMA.
template <int OP, int NC, int ACT, int DM>
__device__ __forceinline__ f32x4v wave_tile(const GemmArgs& g, int r0, int c0, int k0, int nch,
                                            int lane, uint32_t step, float* asum,
                                            f32x4v acc = {0.f, 0.f, 0.f, 0.f}) {
  const int r = lane & 15, q = lane >> 4;
  float a[NC][4], b[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c)
    load_ab<OP, ACT, DM>(g, r0, c0, r, k0 + 16 * c + 4 * q, c < nch, step, a[c], b[c]);
#ifdef PCADV_STAMPS
  if (OP != OP_BWD_WEIGHT) {
    asm volatile("" ::: "memory");
    LSTAMP(g, 5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LSTAMP(g, 4);
  }
#endif
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc = mfma16(a[c][j], b[c][j], acc);
      s += a[c][j];
    }
  }
  *asum = s;
  return acc;
}

// Backward-data tile with dz stored as is (ACT_NONE, DM_NONE, N % 4 == 0):
// the B operand W[n][c0 + r] is a column walk of W, which as one 4-byte load
// per MFMA costs a vector-memory instruction per 256 bytes (issue-bound at the
// start of a launch: tools/lin_stamps.py).  The wave instead fetches its
// 16*NC x 16 block of W as 16-byte row pieces, parks it in its own LDS
// region and reads the fragments from there.  Same operands, same MFMA order:
// bitwise the result of wave_tile<OP_BWD_DATA>.
constexpr int BT_S = 20;                // LDS row stride (floats): conflict-free fragment reads
constexpr int BT_WAVE = 16 * SPLITC * BT_S;
constexpr int BT_MAXS = 8;              // waves per block with an LDS region
template <int NC>
__device__ __forceinline__ f32x4v wave_tile_bdt(const GemmArgs& g, int r0, int c0, int k0, int nch,
                                                int lane, float* bt, f32x4v acc) {
  const int r = lane & 15, q = lane >> 4;
  const int m = r0 + r;
  float a[NC][4];
  f32x4v wv[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int kk = k0 + 16 * c + 4 * q;
    const bool va = c < nch && m < g.M && kk < g.N;
    const f32x4v av = *reinterpret_cast<const f32x4v*>(g.dy + (size_t)(va ? m : 0) * g.N +
                                                       (va ? kk : 0));
#pragma unroll
    for (int j = 0; j < 4; ++j) a[c][j] = va ? av[j] : 0.f;
    // W rows n = k0 + 16c + lane/4, columns c0 + 4 (lane & 3) .. + 3
    const int n = k0 + 16 * c + (lane >> 2), kc = c0 + 4 * (lane & 3);
    const bool vb = c < nch && n < g.N && kc < g.K;
    const f32x4v w = *reinterpret_cast<const f32x4v*>(g.w + (size_t)(vb ? n : 0) * g.K +
                                                      (vb ? kc : 0));
    wv[c] = vb ? w : f32x4v{0.f, 0.f, 0.f, 0.f};
  }
#ifdef PCADV_STAMPS
  asm volatile("" ::: "memory");
  LSTAMP(g, 5);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  LSTAMP(g, 4);
#endif
#pragma unroll
  for (int c = 0; c < NC; ++c)
    *reinterpret_cast<f32x4v*>(bt + (16 * c + (lane >> 2)) * BT_S + 4 * (lane & 3)) = wv[c];
  // the wave's own lanes read what the others wrote
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = mfma16(a[c][j], bt[(16 * c + 4 * q + j) * BT_S + r], acc);
  }
  // the region is rewritten by the next round of the same wave
  __builtin_amdgcn_wave_barrier();
  return acc;
}

// Split-reduction job (forward, backward-data): block = one 16x16 tile, wave w
// takes reduction slice w.  Tiles are numbered row-major over (rows, cols).
// bt: LDS regions for wave_tile_bdt (backward data, dz as is), or nullptr.
template <int OP, int ACT, int DM>
__device__ void split_job(const GemmArgs& g, int tile, int rows, int cols, int R, int S, int L,
                          float* red, float* bt = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t step = DM == DM_RNG ? (uint32_t)*g.drop.step : 0u;
  const int ctiles = (cols + 15) / 16;
  const int r0 = (tile / ctiles) * 16, c0 = (tile % ctiles) * 16;
  const int k0 = wave * L;
  // a slice longer than 16 * SPLITC (reductions > 1024) runs in rounds
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int base = 0; base < L; base += 16 * SPLITC) {
    const int kb = k0 + base;
    int nch = 0;
    if (kb < R) nch = min(min(L - base, 16 * SPLITC), R - kb + 15) / 16;
    float s;
    if (OP == OP_BWD_DATA && ACT == ACT_NONE && DM == DM_NONE && bt)
      acc = wave_tile_bdt<SPLITC>(g, r0, c0, kb, nch, lane, bt + wave * BT_WAVE, acc);
    else
      acc = wave_tile<OP, SPLITC, ACT, DM>(g, r0, c0, kb, nch, lane, step, &s, acc);
  }
  LSTAMP(g, 1);
  const int col = lane & 15, q = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) red[wave * 256 + (4 * q + j) * 16 + col] = acc[j];
  __syncthreads();
  LSTAMP(g, 2);
  for (int e = tid; e < 256; e += 64 * S) {
    const int row = e >> 4, cc = e & 15;
    float v = 0.f;
    for (int w = 0; w < S; ++w) v += red[w * 256 + e];
    const int m = r0 + row, n = c0 + cc;
    if (m < rows && n < cols) {
      if (OP == OP_FWD) {
        const size_t i = (size_t)m * g.N + n;
        v += g.b[n];
        if (DM != DM_NONE) {
          const float sc = drop_scale<DM>(g, i, m, n, step);
          v *= sc;
          // the drawn mask, for a backward that should not redraw it
          if (DM == DM_RNG && g.mask_out) g.mask_out[i] = sc != 0.f ? 1.f : 0.f;
        }
        float o = act_fwd(v, ACT);
        // STNkd / STN3d add the flattened identity (models/pointnet.py:38-41,74-77)
        if (g.diag && n % (g.diag + 1) == 0) o += 1.f;
        g.y[i] = o;
      } else {
        const size_t i = (size_t)m * g.K + n;
        if (g.ox_act != ACT_NONE) v *= act_bwd(g.x[i], g.ox_act);
        if (g.ox_mask) v *= g.ox_mask[i] * g.ox_keep;
        g.dx[i] = v;
        if (OP == OP_BWD_DATA && g.chain_out) bt[e] = v;
      }
    }
  }
  if (OP == OP_BWD_DATA && g.chain_out && r0 >= g.chain_row0) {
    // this tile's share of dx[rows] W'[c0 .. c0 + 16][:]: 16 x chain_n on
    // 16x16x4 MFMAs (exact f32), k = the tile's 16 columns in order; the tile
    // sits in bt[] (rows or columns past the matrix are zero)
    for (int e = tid; e < 256; e += 64 * S) {
      const int row = e >> 4, cc = e & 15;
      if (!(r0 + row < rows && c0 + cc < cols)) bt[e] = 0.f;
    }
    __syncthreads();
    const int nt = (g.chain_n + 15) / 16, r = lane & 15;
    if (wave < nt) {
      const int j = 16 * wave + r;
      f32x4v acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int k = 4 * s4 + q;
        const bool vb = j < g.chain_n && c0 + k < cols;
        const float wv = g.chain_w[(size_t)(vb ? c0 + k : 0) * g.chain_n + (vb ? j : 0)];
        acc2 = mfma16(bt[r * 16 + k], vb ? wv : 0.f, acc2);
      }
      const int nrc = g.M - g.chain_row0;
      float* out = g.chain_out + ((size_t)(c0 / 16) * nrc + (r0 - g.chain_row0)) * g.chain_n;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = 4 * q + v;
        if (r0 + row < rows && j < g.chain_n) out[(size_t)row * g.chain_n + j] = acc2[v];
      }
    }
  }
}

// Weight-gradient job: every wave owns one 16x16 tile of dw (rows n, cols k)
// and the full reduction over the m_w rows; k-tile 0 also produces db.
template <int ACT, int DM>
__device__ void weight_job(const GemmArgs& g, int tile, int ntiles_total) {
  const int lane = threadIdx.x & 63;
  if (tile >= ntiles_total) return;
  if constexpr (ACT == ACT_NONE && DM == DM_NONE) {
    // dz stored as is: the shared job code (wgrad.h), bitwise the same as the
    // deferred jobs that ride along the feature backward
    const WgradJob j{g.dy, g.x, g.dw, g.db, g.N, g.K, g.m_w, 0};
    wgrad_wave(j, tile, lane);
    return;
  }
  const uint32_t step = DM == DM_RNG ? (uint32_t)*g.drop.step : 0u;
  const int ctiles = (g.K + 15) / 16;
  const int r0 = (tile / ctiles) * 16, c0 = (tile % ctiles) * 16;
  const int nch = (g.m_w + 15) / 16;
  float s;
  // the load count follows the chunk count (m_w <= 64 at B = 32: half the loads)
  const f32x4v acc = nch <= MAXC / 2
                         ? wave_tile<OP_BWD_WEIGHT, MAXC / 2, ACT, DM>(g, r0, c0, 0, nch, lane, step, &s)
                         : wave_tile<OP_BWD_WEIGHT, MAXC, ACT, DM>(g, r0, c0, 0, nch, lane, step, &s);
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

template <int ACT, int DM>
__global__ void __launch_bounds__(1024)
k_linear_fwd(GemmArgs g, int S, int L) {
  __shared__ float red[16 * 256];
  kernarg_prefetch(g.x, g.w, g.b, g.y, g.M, g.N, g.K, g.diag, S, L);
  if (DM != DM_NONE) kernarg_prefetch(g.drop.mask, g.drop.step, g.drop.seed, g.drop.p, g.mask_out);
  LSTAMP(g, 0);
  split_job<OP_FWD, ACT, DM>(g, blockIdx.x, g.M, g.N, g.K, S, L, red);
  LSTAMP(g, 3);
}

// Independent work that rides along a backward launch (saves a dependent
// launch): a second weight-gradient job (no activation / dropout), and a
// fixed-order sum of partial slabs: red_dst[j] = sum_s red_src[s * red_n + j].
struct BwdExtra {
  WgradJob job[LB_MAXJOBS];  // .tiles = this job's blocks (block mode) or wave tiles
  int njobs;
  const float* red_src;
  float* red_dst;
  int red_n, red_cnt, red_ld;
  FinAdam adam;
  int nba_g, nba_d;  // Adam blocks over the generator's range, then the discriminator
};

// Adam over n floats of (p, m, v, g) on blocks [0, nb): one float4 per thread
// and pass, every load of a pass issued before its updates (adam_elem: the
// arithmetic of every other Adam of the library, so bitwise theirs)
__device__ void adam_span(int b, int nb, float* p, float* m, float* v, const float* g, int64_t n,
                          const AdamHp& h) {
  const int64_t n4 = n / 4, stride = (int64_t)nb * blockDim.x;
  for (int64_t i = (int64_t)b * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 p4 = reinterpret_cast<const f32x4*>(p)[i], m4 = reinterpret_cast<const f32x4*>(m)[i];
    f32x4 v4 = reinterpret_cast<const f32x4*>(v)[i];
    const f32x4 g4 = reinterpret_cast<const f32x4*>(g)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pp = p4[e], mm = m4[e], vv = v4[e];
      adam_elem(pp, g4[e], mm, vv, h);
      p4[e] = pp;
      m4[e] = mm;
      v4[e] = vv;
    }
    reinterpret_cast<f32x4*>(p)[i] = p4;
    reinterpret_cast<f32x4*>(m)[i] = m4;
    reinterpret_cast<f32x4*>(v)[i] = v4;
  }
  if (b == 0 && (int64_t)threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    adam_elem(p[i], g[i], m[i], v[i], h);
  }
}

// The weight-gradient blocks of a launch: the block-level LDS-staged form
// (wgrad.h) where the layer allows it, else one tile per wave.
static bool wgrad_block_mode(int act, int dm, int N, int K, int S) {
  return act == ACT_NONE && dm == DM_NONE && (N & 3) == 0 && (K & 3) == 0 && S >= WGB_MIN_WAVES;
}

// LDS of the <ACT_NONE, DM_NONE> instance: the backward-data blocks' W regions
// + partials, or a weight-gradient block's staged operands
constexpr int LB_RED = 16 * 256;
constexpr int LB_LDS = BT_MAXS * BT_WAVE + LB_RED > WGB_LDS_FLOATS ? BT_MAXS * BT_WAVE + LB_RED
                                                                   : WGB_LDS_FLOATS;

// blocks [0, nbx): dx tiles (split over S waves); then dw tiles (S per block,
// or one 64x32 region per block in block mode, wmode bit 0); then the extra
// weight tiles (block mode: wmode bit 1); then the slab reduction
template <int ACT, int DM>
__global__ void __launch_bounds__(1024)
k_linear_bwd(GemmArgs g, int S, int L, int nbx, int nwt, BwdExtra ex, int blk0, int wmode) {
  kernarg_prefetch(g.x, g.w, g.dy, g.dx, g.dw, g.db, g.M, g.N, g.K, g.m_w, g.ox_act, g.ox_mask,
                   g.ox_keep, S, L, nbx, nwt, blk0, ex.njobs, ex.red_src, ex.red_dst, ex.red_n,
                   ex.red_cnt, ex.red_ld, wmode, g.chain_out, g.chain_w, g.chain_row0, g.chain_n);
  if (ACT != ACT_NONE) kernarg_prefetch(g.yact);
  if (DM != DM_NONE) kernarg_prefetch(g.drop.mask, g.drop.step, g.drop.seed, g.drop.p);
  constexpr bool FAST = ACT == ACT_NONE && DM == DM_NONE;
  __shared__ __attribute__((aligned(16))) float lds[FAST ? LB_LDS : LB_RED];
  float* red = FAST ? lds + BT_MAXS * BT_WAVE : lds;
  const int nbw = (wmode & 1) ? wgrad_regions(g.N, g.K) : (nwt + S - 1) / S;
  int b = blockIdx.x + blk0;
  LSTAMP(g, 0);
  if (b < nbx) {
    const bool use_bt = FAST && S <= BT_MAXS && (g.N & 3) == 0;
    split_job<OP_BWD_DATA, ACT, DM>(g, b, g.M, g.K, g.N, S, L, red, use_bt ? lds : nullptr);
    LSTAMP(g, 3);
    return;
  }
  b -= nbx;
  if (b < nbw) {
    if (FAST && (wmode & 1)) {
      if (nwt > 0) wgrad_region(WgradJob{g.dy, g.x, g.dw, g.db, g.N, g.K, g.m_w, 0}, b, lds, S);
    } else {
      weight_job<ACT, DM>(g, b * S + (threadIdx.x >> 6), nwt);
    }
    LSTAMP(g, 3);
    return;
  }
  b -= nbw;
  // the extra jobs (block mode: one region per block, wmode bit 1; else one
  // tile per wave)
  for (int i = 0; i < LB_MAXJOBS; ++i) {
    if (i >= ex.njobs) break;
    if (b < ex.job[i].tiles) {
      if (FAST && (wmode & 2)) wgrad_region(ex.job[i], b, lds, S);
      else if (b * S + (int)(threadIdx.x >> 6) < ((ex.job[i].N + 15) / 16) * ((ex.job[i].K + 15) / 16))
        wgrad_wave(ex.job[i], b * S + (threadIdx.x >> 6), (int)threadIdx.x & 63);
      LSTAMP(g, 3);
      return;
    }
    b -= ex.job[i].tiles;
  }
  const int nred = ex.red_n > 0 ? (ex.red_n + 64 * S - 1) / (64 * S) : 0;
  if (b < nred) {
    const int j = b * 64 * S + threadIdx.x;
    if (j < ex.red_n) {
      float acc = 0.f;
      for (int s = 0; s < ex.red_cnt; ++s) acc += ex.red_src[(size_t)s * ex.red_ld + j];
      ex.red_dst[j] = acc;
    }
    LSTAMP(g, 3);
    return;
  }
  b -= nred;
  // Adam of the parameters whose gradients were final before this launch
  const FinAdam& fa = ex.adam;
  if (b < ex.nba_g) {
    const AdamHp h = adam_hp(fa.step_count, fa.step_offset, fa.b1, fa.b2, fa.eps, fa.lr_g);
    adam_span(b, ex.nba_g, fa.gp + fa.g_rest0, fa.gm + fa.g_rest0, fa.gv + fa.g_rest0,
              fa.gg + fa.g_rest0, fa.g_n - fa.g_rest0, h);
  } else if (b - ex.nba_g < ex.nba_d) {
    const AdamHp h = adam_hp(fa.step_count, fa.step_offset, fa.b1, fa.b2, fa.eps, fa.lr_d);
    adam_span(b - ex.nba_g, ex.nba_d, fa.dp, fa.dm, fa.dv, fa.dg, fa.d_n, h);
  }
  LSTAMP(g, 3);
}

// host-side dispatch over the (activation, dropout-source) instantiations
template <template <int, int> class K, typename... Args>
static void launch_variant(int act, int dm, dim3 grid, dim3 block, hipStream_t s, Args... args) {
#define PC_VARIANT(A, D)                                                               \
  if (act == A && dm == D) {                                                           \
    auto kfn_ = K<A, D>::fn;                                                           \
    hipLaunchKernelGGL(kfn_, grid, block, 0, s, args...);                              \
    return;                                                                            \
  }
  PC_VARIANT(ACT_NONE, DM_NONE) PC_VARIANT(ACT_NONE, DM_MASK) PC_VARIANT(ACT_NONE, DM_RNG)
  PC_VARIANT(ACT_RELU, DM_NONE) PC_VARIANT(ACT_RELU, DM_MASK) PC_VARIANT(ACT_RELU, DM_RNG)
  PC_VARIANT(ACT_LRELU, DM_NONE) PC_VARIANT(ACT_LRELU, DM_MASK) PC_VARIANT(ACT_LRELU, DM_RNG)
#undef PC_VARIANT
}

template <int A, int D>
struct FwdK {
  static constexpr auto fn = k_linear_fwd<A, D>;
};
template <int A, int D>
struct BwdK {
  static constexpr auto fn = k_linear_bwd<A, D>;
};

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
                      float p, hipStream_t s, int add_identity_k, float* mask_out,
                      int row_split, int row_off_lo, int row_off_hi) {
  PC_REQUIRE(M > 0 && N > 0 && K > 0 && K % 4 == 0, "linear_fwd: bad shape M=%d N=%d K=%d", M, N,
             K);
  PC_REQUIRE(add_identity_k == 0 || add_identity_k * add_identity_k == N,
             "linear_fwd: identity of size %d does not match %d outputs", add_identity_k, N);
  GemmArgs g{};
  g.x = x; g.w = w; g.b = b; g.y = y; g.act = act; g.diag = add_identity_k;
  g.mask_out = mask_out;
  g.drop = DropSpec{mask, step, seed, p, row_split, row_off_lo, row_off_hi};
  g.M = M; g.N = N; g.K = K;
  int S, L;
  split_cfg(K, &S, &L);
  PC_REQUIRE(act == ACT_NONE || act == ACT_RELU || act == ACT_LRELU, "linear_fwd: bad act %d", act);
  const int tiles = ((M + 15) / 16) * ((N + 15) / 16);
  g.stamp_slot = next_stamp_slot();
  launch_variant<FwdK>(act, drop_mode(g.drop), dim3(tiles), dim3(64 * S), s, g, S, L);
  PC_HIP_CHECK_LAUNCH("k_linear_fwd");
  return PCADV_OK;
}

int launch_linear_bwd(const float* dy, const float* y, int act, const float* mask,
                      const int32_t* step, uint64_t seed, float p, const float* x, const float* w,
                      float* dx, float* dw, float* db, int M, int m_w, int N, int K,
                      hipStream_t s, const LinBwdExtra* extra) {
  // the weight-gradient rows: any number with dz as is (wgrad.h forms), at
  // most 16 MAXC when an activation or dropout applies on the fly
  const bool dz_as_is = act == ACT_NONE && !mask && !step;
  PC_REQUIRE(M > 0 && N > 0 && K > 0 && K % 4 == 0 && m_w >= 0 && m_w <= M &&
                 (dz_as_is || !dw || m_w <= 16 * MAXC),
             "linear_bwd: bad shape M=%d m_w=%d N=%d K=%d", M, m_w, N, K);
  GemmArgs g{};
  g.x = x; g.w = w; g.dy = dy; g.yact = y; g.act = act;
  g.drop = DropSpec{mask, step, seed, p, 0, 0, 0};
  g.dx = dx; g.dw = dw; g.db = db;
  g.M = M; g.N = N; g.K = K; g.m_w = m_w;
  if (extra) {
    PC_REQUIRE(extra->dx_act == ACT_NONE || extra->dx_act == ACT_RELU || extra->dx_act == ACT_LRELU,
               "linear_bwd: bad dx_act %d", extra->dx_act);
    PC_REQUIRE(!(extra->dx_act != ACT_NONE || extra->dx_mask) || (dx && x),
               "linear_bwd: the dx output mask needs dx and the layer input x");
    g.ox_act = extra->dx_act;
    g.ox_mask = extra->dx_mask;
    g.ox_keep = extra->dx_keep;
    g.chain_w = extra->chain_w;
    g.chain_out = extra->chain_out;
    g.chain_row0 = extra->chain_row0;
    g.chain_n = extra->chain_n;
  }
  int S, L;
  split_cfg(N, &S, &L);
  if (g.chain_out) {
    // the tile product runs in the backward-data blocks' LDS regions, one
    // 16-column output tile per wave, on row tiles that start at chain_row0
    PC_REQUIRE(dx && g.chain_w && dz_as_is && (N & 3) == 0 && S <= BT_MAXS && g.chain_n > 0 &&
                   g.chain_n <= 16 * S && g.chain_row0 >= 0 && g.chain_row0 < M &&
                   g.chain_row0 % 16 == 0,
               "linear_bwd: bad chained product (n=%d row0=%d S=%d)", g.chain_n, g.chain_row0, S);
  }
  const int nbx = dx ? ((M + 15) / 16) * ((K + 15) / 16) : 0;
  const int nwt = dw ? ((N + 15) / 16) * ((K + 15) / 16) : 0;
  const int dm = drop_mode(g.drop);
  int wmode = 0;
  if (nwt > 0 && wgrad_block_mode(act, dm, N, K, S)) wmode |= 1;
  const int nbw = nwt == 0 ? 0 : (wmode & 1) ? wgrad_regions(N, K) : (nwt + S - 1) / S;
  BwdExtra ex{};
  int nbe = 0;
  if (extra) {
    PC_REQUIRE(extra->njobs >= 0 && extra->njobs <= LB_MAXJOBS, "linear_bwd: %d extra jobs",
               extra->njobs);
    // extra jobs in block mode when this launch's blocks allow it (all of them or none)
    bool blk = S >= WGB_MIN_WAVES;
    for (int i = 0; i < extra->njobs; ++i) {
      const LinBwdJob& e = extra->job[i];
      PC_REQUIRE(e.dz && e.x && e.dw && e.N > 0 && e.K > 0 && e.m_w > 0 && e.K % 4 == 0,
                 "linear_bwd: bad extra weight job %d (m_w=%d N=%d K=%d)", i, e.m_w, e.N, e.K);
      blk = blk && (e.N & 3) == 0;
    }
    if (blk && extra->njobs > 0) wmode |= 2;
    ex.njobs = extra->njobs;
    for (int i = 0; i < extra->njobs; ++i) {
      const LinBwdJob& e = extra->job[i];
      WgradJob& j = ex.job[i];
      j.dz = e.dz; j.x = e.x; j.dw = e.dw; j.db = e.db;
      j.N = e.N; j.K = e.K; j.m_w = e.m_w;
      const int tiles = ((e.N + 15) / 16) * ((e.K + 15) / 16);
      j.tiles = blk ? wgrad_regions(e.N, e.K) : (tiles + S - 1) / S;  // blocks of this job
      nbe += j.tiles;
    }
    if (extra->red_src) {
      PC_REQUIRE(extra->red_dst && extra->red_n > 0 && extra->red_cnt > 0 &&
                     (extra->red_ld == 0 || extra->red_ld >= extra->red_n),
                 "linear_bwd: bad extra reduction");
      ex.red_src = extra->red_src;
      ex.red_dst = extra->red_dst;
      ex.red_n = extra->red_n;
      ex.red_cnt = extra->red_cnt;
      ex.red_ld = extra->red_ld ? extra->red_ld : extra->red_n;
      nbe += (ex.red_n + 64 * S - 1) / (64 * S);
    }
    if (extra->adam.on) {
      const FinAdam& fa = extra->adam;
      PC_REQUIRE(fa.gp && fa.gm && fa.gv && fa.gg && fa.step_count && fa.g_n >= fa.g_rest0 &&
                     fa.g_rest0 % 4 == 0 && (fa.d_n == 0 || (fa.dp && fa.dm && fa.dv && fa.dg)),
                 "linear_bwd: bad Adam ranges");
      ex.adam = fa;
      const int64_t per = (int64_t)64 * S * 4;  // floats per block and pass
      ex.nba_g = (int)((fa.g_n - fa.g_rest0 + per - 1) / per);
      ex.nba_d = (int)((fa.d_n + per - 1) / per);
      nbe += ex.nba_g + ex.nba_d;
    }
  }
  if (nbx + nbw + nbe == 0) return PCADV_OK;
  PC_REQUIRE(act == ACT_NONE || act == ACT_RELU || act == ACT_LRELU, "linear_bwd: bad act %d", act);
  g.stamp_slot = next_stamp_slot();
  launch_variant<BwdK>(act, dm, dim3(nbx + nbw + nbe), dim3(64 * S), s, g, S, L, nbx, nwt, ex, 0,
                       wmode);
  PC_HIP_CHECK_LAUNCH("k_linear_bwd");
  return PCADV_OK;
}

}  // namespace pcadv

// PointNetfeat backward on gfx950: autograd of models/pointnet.py:115-130.
//
// The max-pool has no ReLU before it (pointnet.py:128-129), so channel o of
// cloud c sends its whole gradient to the single point gidx[c][o]:
//   dW4[o,:] = sum_c g[c,o] x3[c, gidx[c,o], :]            (k_feat_bwd_chunk, trailing workgroups)
//   dX3[c,n,:] = sum_{o: gidx[c,o]=n} g[c,o] W4[o,:]         (k_feat_bwd_chunk)
// Only points that are the argmax of some channel ("active" points, ~1/4 of a
// cloud) carry gradient into conv3..conv1, so k_feat_bwd_chunk compacts them
// and runs the conv3/conv2/conv1 backward (f32 MFMA) on active rows only.
//
// k_feat_bwd_chunk, one workgroup per (cloud, 128-point chunk), 2 per CU:
//   1. the channels whose argmax falls in the chunk ("hits"), keyed (row, o) and
//      sorted by rank counting, so each row's hits are contiguous and in
//      increasing o (fixed summation order -> bitwise reproducible);
//   2. active rows compacted;
//   3. per batch of 32 active rows: recompute x1/x2 from the points, dX3 rows from the sorted
//      hits (loads of W4 rows issued back to back) with the conv3 ReLU mask,
//      dX2 = dZ3 W3 and dX1 = dZ2 W2 on v_mfma_f32_16x16x4_f32 (one 16x16 tile
//      per wave), weight gradients on v_mfma_f32_32x32x2_f32.
// Each workgroup writes its weight-gradient partials to its own slab;
// k_feat_bwd_finish sums the slabs in a fixed order (no atomics).
#include "common.h"
#include "feat_sort.h"

namespace pcadv {

constexpr int BW_PCH = 128;   // points per workgroup (chunk)
constexpr int BW_RB = 32;     // active rows per batch
constexpr int BW_MAXO = 1024; // channels of the pooled layer
constexpr int BW_T = 512;     // threads per workgroup (8 waves), 2 workgroups per CU
constexpr int SLAB = 12736;   // dW1 192 | db1 64 | dW2 4096 | db2 64 | dW3 8192 | db3 128
constexpr int SL_DW1 = 0, SL_DB1 = 192, SL_DW2 = 256, SL_DB2 = 4352, SL_DW3 = 4416, SL_DB3 = 12608;
constexpr int SZ3 = 130;      // LDS stride of 128-wide rows (= 2 mod 32: 16x16x4 row reads
constexpr int SZ2 = 66;       //  and 32x32x2 column reads are both conflict-free)

typedef float f32x4m __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4m mfma16(float a, float b, f32x4m c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int BW_G = 12;      // hit groups of the dZ3 gather: half-waves of waves 2-7 (4 columns per lane)
constexpr int BW_RBG = (BW_RB + BW_G - 1) / BW_G;  // batch rows per gather group (mask / combine)
constexpr int BW_GD = 8;      // W4 rows in flight per gather lane
struct BwdLds {
  union {
    struct {
      int key[BW_MAXO];      // o of each hit, grouped by row (arbitrary order in a row)
      float hg[BW_MAXO];     // g of each hit, same order
    };
    alignas(16) float bnd[BW_G][128];  // group g's partial dZ3 sums of its cut row (phase b)
  };
  int so[BW_MAXO];           // o of each hit, sorted by (row, o)
  float sg[BW_MAXO];         // g, same order
  int rcnt[BW_PCH];          // hits per row of the chunk
  int fill[BW_PCH];          // placement cursor per row
  int roff[BW_PCH];          // first hit of each row (exclusive scan of rcnt)
  int wsum[2], wact[2];
  int rows_list[BW_PCH];     // compact slot -> row
  int hoff[BW_PCH + 4];      // first sorted hit of each compact slot; hoff[nact] = nhits
  alignas(16) int bnd_row[BW_G];  // batch row whose hits group g continued (or -1)
  alignas(16) float dz3[BW_RB * SZ3];
  alignas(16) float x2[BW_RB * S64];   // recomputed conv2 output (f32, as the forward)
  alignas(16) float x1[BW_RB * S64];   // recomputed conv1 output
  alignas(16) float dz2[BW_RB * SZ2];
  alignas(16) float dz1[BW_RB * SZ2];
  alignas(16) float pts[BW_RB * 4];
};

static_assert(FS_PCH == BW_PCH && FS_MAXO == BW_MAXO && FS_T == BW_T, "feat_sort.h geometry");

// Adam over the parameters whose gradients are final before the feature
// backward: the generator from fc1 on (segment 0) and the discriminator
// (segment 1), in trailing workgroups of k_feat_bwd_chunk (NT = BW_T threads);
// V4 float4 per thread and pass, blocks [0, nb0) on segment 0.
#ifndef PCADV_FIN_ADAM_V4
#define PCADV_FIN_ADAM_V4 4
#endif
#ifndef PCADV_TRAIL_ADAM_FIRST
#define PCADV_TRAIL_ADAM_FIRST 0
#endif
constexpr int FIN_ADAM_V4 = PCADV_FIN_ADAM_V4;  // float4 per thread in the chunk launch's Adam workgroups
template <int NT, int V4>
__device__ void adam_range(int b, int nb, float* p, float* m, float* v, const float* g, int64_t n,
                           float lr, const FinAdam& fa) {
  const AdamHp h = adam_hp(fa.step_count, fa.step_offset, fa.b1, fa.b2, fa.eps, lr);
  const int64_t n4 = n / 4;
  // V4 float4 per thread, all loads issued before any update: one
  // memory round trip per pass
  const int64_t stride = (int64_t)nb * NT;
  for (int64_t i0 = (int64_t)b * NT + threadIdx.x; i0 < n4; i0 += stride * V4) {
    f32x4 p4[V4], g4[V4], m4[V4], v4[V4];
#pragma unroll
    for (int u = 0; u < V4; ++u) {
      const int64_t i = i0 + u * stride < n4 ? i0 + u * stride : i0;  // clamped, not stored
      p4[u] = reinterpret_cast<f32x4*>(p)[i];
      g4[u] = reinterpret_cast<const f32x4*>(g)[i];
      m4[u] = reinterpret_cast<f32x4*>(m)[i];
      v4[u] = reinterpret_cast<f32x4*>(v)[i];
    }
#pragma unroll
    for (int u = 0; u < V4; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n4) continue;
      float pp[4] = {p4[u].x, p4[u].y, p4[u].z, p4[u].w};
      float mm[4] = {m4[u].x, m4[u].y, m4[u].z, m4[u].w};
      float vv[4] = {v4[u].x, v4[u].y, v4[u].z, v4[u].w};
      const float gg[4] = {g4[u].x, g4[u].y, g4[u].z, g4[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) adam_elem(pp[e], gg[e], mm[e], vv[e], h);
      reinterpret_cast<f32x4*>(p)[i] = f32x4{pp[0], pp[1], pp[2], pp[3]};
      reinterpret_cast<f32x4*>(m)[i] = f32x4{mm[0], mm[1], mm[2], mm[3]};
      reinterpret_cast<f32x4*>(v)[i] = f32x4{vv[0], vv[1], vv[2], vv[3]};
    }
  }
  if (b == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    adam_elem(p[i], g[i], m[i], v[i], h);
  }
}
template <int NT, int V4>
__device__ void adam_block(int blk, int nb0, int nb1, const FinAdam& fa) {
  if (blk < nb0)
    adam_range<NT, V4>(blk, nb0, fa.gp + fa.g_rest0, fa.gm + fa.g_rest0, fa.gv + fa.g_rest0,
                       fa.gg + fa.g_rest0, fa.g_n - fa.g_rest0, fa.lr_g, fa);
  else
    adam_range<NT, V4>(blk - nb0, nb1, fa.dp, fa.dm, fa.dv, fa.dg, fa.d_n, fa.lr_d, fa);
}
static int fin_adam_blocks(int64_t n, int nt, int v4) {
  int64_t b = (n / 4 + (int64_t)nt * v4 - 1) / ((int64_t)nt * v4);
  return (int)(b < 1 ? 1 : b);
}

// dW4[o,:] = sum_c g[c,o] x3[c, gidx[c,o], :];  db4[o] = sum_c g[c,o].
// In trailing workgroups of k_feat_bwd_chunk (it needs only dg, gidx and x3,
// all final before that launch): NW waves per workgroup, DW4_WPC waves per
// channel, each summing a contiguous share of the clouds in cloud order, the
// shares then added in order (fixed).
// Lanes hold two of the 128 columns.  Per group of 64 clouds, lane c fetches
// (g, gidx) of cloud c once and the row addresses are broadcast with
// v_readlane (scalar base + lane offset), so the row loads are all in flight
// together: two memory round trips per wave.
constexpr int DW4_WPC = 2;  // waves per channel
// XB: x3 is bf16 (bf16 mode's forward store), two columns in one 4-B load
template <int NW, bool XB>
__device__ void dw4_block(int blk, float4 (*part)[64], const float* __restrict__ dg,
                          const int32_t* __restrict__ gidx, int C, int N, int O,
                          const float* __restrict__ x3, float* __restrict__ dw4,
                          float* __restrict__ db4) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int o = blk * (NW / DW4_WPC) + wave / DW4_WPC, qq = wave % DW4_WPC;
  const int ca = C * qq / DW4_WPC, cb = C * (qq + 1) / DW4_WPC;
  float ax = 0.f, ay = 0.f, ab = 0.f;
  if (o < O) {
    for (int c0 = ca; c0 < cb; c0 += 64) {
      const int cl = c0 + lane, cnt = min(64, cb - c0);
      const bool vl = lane < cnt;
      const float gl = vl ? dg[(size_t)cl * O + o] : 0.f;
      const int nl = vl ? gidx[(size_t)cl * O + o] : 0;
      constexpr int U = 16;
      for (int u0 = 0; u0 < cnt; u0 += U) {
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int cu = min(u0 + u, cnt - 1);  // clamped: loads past cnt are discarded
          const int n = __builtin_amdgcn_readlane(nl, cu);
          const size_t off = ((size_t)(c0 + cu) * N + n) * 128 + 2 * lane;
          if constexpr (XB) {
            const uint32_t b = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const __bf16*>(x3) + off);
            v[u] = make_float2(__uint_as_float(b << 16), __uint_as_float(b & 0xffff0000u));
          } else {
            v[u] = *reinterpret_cast<const float2*>(x3 + off);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u0 + u < cnt) {
            const float g = __builtin_bit_cast(
                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, gl), u0 + u));
            ax = fmaf(g, v[u].x, ax);
            ay = fmaf(g, v[u].y, ay);
            ab += g;
          }
        }
      }
    }
  }
  part[wave][lane] = make_float4(ax, ay, ab, 0.f);
  __syncthreads();
  if (qq == 0 && o < O) {
    float4 t = part[wave][lane];
#pragma unroll
    for (int k = 1; k < DW4_WPC; ++k) {
      const float4 p = part[wave + k][lane];
      t.x += p.x;
      t.y += p.y;
      t.z += p.z;
    }
    *reinterpret_cast<float2*>(dw4 + (size_t)o * 128 + 2 * lane) = make_float2(t.x, t.y);
    if (lane == 0) db4[o] = t.z;
  }
}


#ifdef PCADV_STAMPS
// diagnostic build only: the stamps of a launch given no stamps buffer (the
// chunk launch inside a step): [y * gridDim.x + x][32], trailing workgroups
// stamp slot 0 (start) and 14 (end) and carry -1 in slot 15
__device__ uint64_t g_chunk_stamps[1024][32];
int chunk_stamps_read(uint64_t* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chunk_stamps), sizeof(g_chunk_stamps)) == hipSuccess
             ? PCADV_OK
             : PCADV_EHIP;
}
#endif

// PRE: phases 1-3 (the hit sort) were done ahead of this launch (feat_sort.h,
// records at sortrec): load them and gather the hits' gradients instead.
// XB: x3 is bf16 (bf16 mode): the conv3 ReLU mask and the dW4 gather read it so
template <bool PRE, bool XB>
__global__ void __launch_bounds__(BW_T, 4)
k_feat_bwd_chunk(const float* __restrict__ dg, const int32_t* __restrict__ gidx, int O,
                 const float* __restrict__ pts_a, const float* __restrict__ pts_b, int split,
                 int N, const float* __restrict__ w1, const float* __restrict__ b1,
                 const float* __restrict__ w2, const float* __restrict__ b2,
                 const float* __restrict__ w3, const float* __restrict__ w4,
                 const float* __restrict__ x3, float* __restrict__ slabs, uint64_t* stamps,
                 const int* __restrict__ sortrec, int nclouds, float* __restrict__ dw4,
                 float* __restrict__ db4, FinAdam fa, int nb_adam0, int nb_adam1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // Workgroup rows past the clouds: work that needs nothing from this launch,
  // the dW4 / db4 gather and the Adam update of the parameters whose gradients
  // are final before it (G from fc1 on, D; not W4, which the chunks read).  They are
  // dispatched last, so they take the CU slots of the chunks that finish first
  // while the two-batch chunks run on.
  if ((int)blockIdx.y >= nclouds) {
#ifdef PCADV_STAMPS
    const size_t wg_ = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    if (!stamps && threadIdx.x == 0 && wg_ < 1024) g_chunk_stamps[wg_][0] = __builtin_amdgcn_s_memrealtime();
#endif
    const int b = ((int)blockIdx.y - nclouds) * (int)gridDim.x + (int)blockIdx.x;
    constexpr int NDW4 = BW_MAXO / (BW_T / 64 / DW4_WPC);
    const int nad = nb_adam0 + nb_adam1;
    const bool is_dw4 = PCADV_TRAIL_ADAM_FIRST ? (b >= nad && b - nad < NDW4) : b < NDW4;
    const int bd = PCADV_TRAIL_ADAM_FIRST ? b - nad : b, ba = PCADV_TRAIL_ADAM_FIRST ? b : b - NDW4;
    if (is_dw4)
      dw4_block<BW_T / 64, XB>(bd, reinterpret_cast<float4(*)[64]>(smem), dg, gidx, nclouds, N, O, x3,
                           dw4, db4);
    else if (ba >= 0 && ba < nad)
      adam_block<BW_T, FIN_ADAM_V4>(ba, nb_adam0, nb_adam1, fa);
#ifdef PCADV_STAMPS
    __syncthreads();
    if (!stamps && threadIdx.x == 0 && wg_ < 1024) {
      g_chunk_stamps[wg_][14] = __builtin_amdgcn_s_memrealtime();
      g_chunk_stamps[wg_][15] = is_dw4 ? -1 : -2;
    }
#endif
    return;
  }
  BwdLds& L = *reinterpret_cast<BwdLds*>(smem);
#ifdef PCADV_STAMPS
  // diagnostic build only: per-workgroup phase timestamps (s_memrealtime, 100 MHz)
  // 32 slots per workgroup: 0-15 by thread 0 (below); 16 + batch by thread 128
  // (wave 2) when its dZ3 gather loop is done; 24 + k: phase a of batch 1
  const size_t wgi_ = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
  uint64_t* st_ = stamps ? stamps + wgi_ * 32 : (wgi_ < 1024 ? g_chunk_stamps[wgi_] : nullptr);
#define BSTAMP(k) do { if (st_ && threadIdx.x == 0 && (k) < 15) st_[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define GSTAMP(k) do { if (st_ && threadIdx.x == 128 && (k) < 8) st_[16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define ASTAMP(k) do { if (st_ && threadIdx.x == 0 && b0 == 0) st_[24 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define BSTAMP(k) do { } while (0)
#define GSTAMP(k) do { } while (0)
#define ASTAMP(k) do { } while (0)
#endif
  BSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y, chunk = blockIdx.x, p0 = chunk * BW_PCH;
  const float* pts = c < split ? pts_a + (size_t)c * N * 3 : pts_b + (size_t)(c - split) * N * 3;

  // wave -> (row tile rt, column tile ct) of the 32 x 64 dX2 / dX1 outputs;
  // its B fragments (16x16x4, k = 4s + q) are re-read from L2 each batch
  const int rt = wave >> 2, ct = wave & 3;
  // buffer loads: 32-bit lane offsets + scalar step offsets, so no 64-bit
  // addresses are kept live across the batch loop
  const __amdgpu_buffer_rsrc_t w3r =
      __builtin_amdgcn_make_buffer_rsrc((void*)w3, (short)0, 128 * 64 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t w2r =
      __builtin_amdgcn_make_buffer_rsrc((void*)w2, (short)0, 64 * 64 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t w4r =
      __builtin_amdgcn_make_buffer_rsrc((void*)w4, (short)0, BW_MAXO * 128 * 4, 0x00020000);
  // this cloud's x3 rows (C x N x 128 f32 < 4 GB: 32-bit offsets from the cloud base)
  constexpr int XE = XB ? 2 : 4;  // bytes per x3 element
  const __amdgpu_buffer_rsrc_t x3r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<const char*>(x3) + (size_t)c * N * 128 * XE), (short)0, N * 128 * XE,
      0x00020000);
  // conv1 weights, fetched up front so they land during the hit sort
  const int ch1 = tid & 63;
  const float w1a = w1[ch1 * 3 + 0], w1b = w1[ch1 * 3 + 1], w1c = w1[ch1 * 3 + 2], b1v = b1[ch1];
  int nact;
  float ptv[2] = {0.f, 0.f};
  if constexpr (PRE) {
    // ---- 1-3 done ahead (feat_sort.h): one round of loads, the fixed-size
    //      record and this cloud's pooled gradients, then g of each sorted hit
    const int* rec = sortrec + ((size_t)c * gridDim.x + chunk) * FS_REC;
    int so_v[2];
    float dg_v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      so_v[u] = rec[FSR_SO + u * BW_T + tid];
      dg_v[u] = dg[(size_t)c * O + u * BW_T + tid];
    }
    int rl_v = 0, ho_v = 0;
    if (tid < BW_PCH) rl_v = rec[FSR_ROWS + tid];
    if (tid <= BW_PCH) ho_v = rec[FSR_HOFF + tid];
    nact = rec[0];
    if (tid < BW_PCH) L.rows_list[tid] = rl_v;
    if (tid <= BW_PCH) L.hoff[tid] = ho_v;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      L.so[u * BW_T + tid] = so_v[u];
      L.hg[u * BW_T + tid] = dg_v[u];  // the cloud's gradient row, indexed by o
    }
    __syncthreads();
    const int nhits = L.hoff[nact];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = u * BW_T + tid;
      if (j < nhits) L.sg[j] = L.hg[L.so[j]];
    }
    if (wave < 2) {  // first batch's points (waves 0-1 hold all 96 coordinates)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = lane + 64 * u, row = e / 3;
        if (e < BW_RB * 3 && row < nact) ptv[u] = pts[(size_t)(p0 + L.rows_list[row]) * 3 + e % 3];
      }
    }
    __syncthreads();
    BSTAMP(3);
  } else {
  if (tid < BW_PCH) {
    L.rcnt[tid] = 0;
    L.fill[tid] = 0;
  }
  __syncthreads();

  // ---- 1. hits: the channels whose argmax falls in this chunk (thread -> 2
  //      channels, kept in registers); count them per row ----------------------
  int hrow[2], hpos[2];
  float hgv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int o = u * BW_T + tid;
    const int a = o < O ? gidx[(size_t)c * O + o] : -1;
    const bool hit = a >= p0 && a < p0 + BW_PCH;
    hrow[u] = hit ? a - p0 : -1;
    hgv[u] = hit ? dg[(size_t)c * O + o] : 0.f;
    if (hit) atomicAdd(&L.rcnt[a - p0], 1);
  }
  __syncthreads();
  BSTAMP(1);

  // ---- 2. active rows (rcnt > 0) compacted in row order; roff / hoff =
  //      exclusive scan of the hit counts (waves 0-1 own one row per lane) ----
  if (wave < 2) {
    const int row = tid, cnt = L.rcnt[row];
    const bool f = cnt > 0;
    int v = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(v, d);
      if (lane >= d) v += t;
    }
    const uint64_t m = __ballot(f);
    if (lane == 63) {
      L.wsum[wave] = v;
      L.wact[wave] = __popcll(m);
    }
    L.roff[row] = v - cnt;  // wave-local for now
  }
  __syncthreads();
  nact = L.wact[0] + L.wact[1];
  const int nhits = L.wsum[0] + L.wsum[1];
  if (wave < 2) {
    const int row = tid;
    const bool f = L.rcnt[row] > 0;
    const uint64_t m = __ballot(f);
    const int slot = (wave ? L.wact[0] : 0) + __popcll(m & ((1ull << lane) - 1ull));
    const int off = L.roff[row] + (wave ? L.wsum[0] : 0);
    L.roff[row] = off;
    if (f) {
      L.rows_list[slot] = row;
      L.hoff[slot] = off;
    }
    if (tid == 0) L.hoff[nact] = nhits;
  }
  // first batch's points, issued now (used after the sort): waves 0-1 each
  // hold all 96 coordinates (element lane + 64 u)
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = lane + 64 * u, row = e / 3;
      if (e < BW_RB * 3 && row < nact) ptv[u] = pts[(size_t)(p0 + L.rows_list[row]) * 3 + e % 3];
    }
  }
  BSTAMP(2);

  // ---- 3. place each hit in its row's segment, then rank it inside the
  //      segment by o: sorted order (row, o), independent of timing ----------
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    hpos[u] = -1;
    if (hrow[u] >= 0) {
      hpos[u] = L.roff[hrow[u]] + atomicAdd(&L.fill[hrow[u]], 1);
      L.key[hpos[u]] = u * BW_T + tid;
      L.hg[hpos[u]] = hgv[u];
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (hrow[u] >= 0) {
      const int o = u * BW_T + tid, s0 = L.roff[hrow[u]], s1 = s0 + L.rcnt[hrow[u]];
      int rank = 0;
      for (int j = s0; j < s1; ++j) rank += L.key[j] < o;
      L.so[s0 + rank] = o;
      L.sg[s0 + rank] = hgv[u];
    }
  }
  __syncthreads();
  BSTAMP(3);
  }  // !PRE

  // register accumulators that live across batches
  f32x16 a_dw3 = {}, a_dw2 = {};
  float acc_w1 = 0.f, acc_b = 0.f;

  for (int b0 = 0; b0 < nact; b0 += BW_RB) {
    // the lane-dependent indices are re-derived in every batch: otherwise each
    // LDS / buffer offset built from them is hoisted out of the batch loop and
    // kept live (or spilled) across it
    int lane_l = lane;
    asm volatile("" : "+v"(lane_l));
    const int lane = lane_l, tid = wave * 64 + lane;
    const int r32 = lane & 31, h = lane >> 5, r16 = lane & 15, q = lane >> 4;
    const int boff = (q * 64 + 16 * ct + r16) * 4;  // this lane's W3 / W2 fragment offset
    const int nb = min(BW_RB, nact - b0);
    const int sb_ = 4 + 5 * (b0 / BW_RB);
    (void)sb_;
    // ---- a | b, side by side: waves 0-1 recompute x1, x2 of the batch rows
    //      (a); waves 2-7 gather the dZ3 rows meanwhile (b), which needs neither.
    if (wave < 2) {
      // a. conv1 (VALU) and conv2 (v_mfma_f32_32x32x2_f32) in the forward's
      //    operation order: bit-identical activations.  Both waves compute all
      //    of x1 and write the same values to the same LDS words, so each wave
      //    only has to order its own accesses (no workgroup barrier).
      f32x4 bf2[8];
      load_bfrag<64>(w2, 32 * wave, lane, bf2);
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // the batch's points: element e = lane + 64 u of 96
        const int e = lane + 64 * u, row = e / 3;
        if (e < BW_RB * 3) L.pts[row * 4 + e % 3] = row < nb ? ptv[u] : 0.f;
      }
      // the next batch's points, in flight until its phase a
      if (b0 + BW_RB < nact) {
        const int nb2 = min(BW_RB, nact - b0 - BW_RB);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int e = lane + 64 * u, row = e / 3;
          if (e < BW_RB * 3)
            ptv[u] = row < nb2 ? pts[(size_t)(p0 + L.rows_list[b0 + BW_RB + row]) * 3 + e % 3] : 0.f;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      ASTAMP(0);
#pragma unroll 8
      for (int rr = 0; rr < BW_RB; ++rr) {
        const f32x4 q4 = *reinterpret_cast<const f32x4*>(&L.pts[rr * 4]);
        L.x1[rr * S64 + lane] = conv1_point(w1a, w1b, w1c, b1v, q4.x, q4.y, q4.z);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      ASTAMP(1);
      f32x16 acc = {};
      acc = mfma_rows_x_wt<64>(L.x1, S64, bf2, acc, lane);
#ifdef PCADV_STAMPS
      asm volatile("s_nop 0" ::"v"(acc[0]), "v"(acc[15]));
#endif
      ASTAMP(2);
      const int col = 32 * wave + r32;
      const float bias = b2[col];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = acc[i] + bias;
        L.x2[acc_row(i, lane) * S64 + col] = v > 0.f ? v : 0.f;
      }
    }
    BSTAMP(sb_);

    // b. dZ3 rows: thread = (column quad cq, group g of 12) on waves 2-7; the
    //    batch's sorted hits are split evenly over the groups whatever their
    //    spread over rows, and each hit's W4 row (512 B) is read by the group's
    //    32 lanes, 16 B each.  A row cut by a group boundary gets the later
    //    groups' partial sums added in group order (fixed order: bitwise
    //    reproducible).
    const int cq = tid & 31, grp = (tid >> 5) - 4;
    uint32_t mask = 0;  // conv3 ReLU mask of rows grp + 12 u (4 columns each)
    if (wave >= 2) {
#pragma unroll
      for (int u = 0; u < BW_RBG; ++u) {
        const int rr = grp + BW_G * u;
        if (rr < nb) {
          const int p = p0 + L.rows_list[b0 + rr];
          f32x4 xv;
          if constexpr (XB) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 b = __builtin_bit_cast(
                u32x2, __builtin_amdgcn_raw_buffer_load_b64(x3r, (p * 128 + 4 * cq) * 2, 0, 0));
            xv = f32x4{__uint_as_float(b.x << 16), __uint_as_float(b.x & 0xffff0000u),
                       __uint_as_float(b.y << 16), __uint_as_float(b.y & 0xffff0000u)};
          } else {
            xv = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(x3r, (p * 128 + 4 * cq) * 4, 0, 0));
          }
          mask |= ((xv.x > 0.f ? 1u : 0u) | (xv.y > 0.f ? 2u : 0u) | (xv.z > 0.f ? 4u : 0u) |
                   (xv.w > 0.f ? 8u : 0u)) << (4 * u);
        }
      }
      const int jb0 = L.hoff[b0], nh = L.hoff[b0 + nb] - jb0;
      const int ja = jb0 + (nh * grp) / BW_G, je = jb0 + (nh * (grp + 1)) / BW_G;
      auto w4_at = [&](int o) {
        return __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(w4r, (o * 128 + 4 * cq) * 4, 0, 0));
      };
      int brow = -1;
      if (ja < je) {
        int s = b0;
        while (L.hoff[s + 1] <= ja) ++s;
        bool head = L.hoff[s] >= ja;  // row s starts inside my range
        if (!head) brow = s - b0;
        int jnext = L.hoff[s + 1];
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        auto flush = [&]() {
          if (head) {  // 8-B aligned rows (SZ3 = 130): two ds_write_b64
            float* d = &L.dz3[(s - b0) * SZ3 + 4 * cq];
            *reinterpret_cast<float2*>(d) = make_float2(acc.x, acc.y);
            *reinterpret_cast<float2*>(d + 2) = make_float2(acc.z, acc.w);
          } else {
            *reinterpret_cast<f32x4*>(&L.bnd[grp][4 * cq]) = acc;
          }
          acc = f32x4{0.f, 0.f, 0.f, 0.f};
          head = true;
          ++s;
          jnext = L.hoff[s + 1];
        };
        auto add = [&](float g, const f32x4& w) {
          acc.x = fmaf(g, w.x, acc.x);
          acc.y = fmaf(g, w.y, acc.y);
          acc.z = fmaf(g, w.z, acc.z);
          acc.w = fmaf(g, w.w, acc.w);
        };
        int j = ja;
        for (; j + BW_GD <= je; j += BW_GD) {
          f32x4 wv[BW_GD];
#pragma unroll
          for (int u = 0; u < BW_GD; ++u) wv[u] = w4_at(L.so[j + u]);
#pragma unroll
          for (int u = 0; u < BW_GD; ++u) {
            while (j + u >= jnext) flush();
            add(L.sg[j + u], wv[u]);
          }
        }
        if (j < je) {
          f32x4 wv[BW_GD];
#pragma unroll
          for (int u = 0; u < BW_GD; ++u)
            wv[u] = j + u < je ? w4_at(L.so[j + u]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int u = 0; u < BW_GD; ++u) {
            if (j + u < je) {
              while (j + u >= jnext) flush();
              add(L.sg[j + u], wv[u]);
            }
          }
        }
        flush();  // the row holding hit je-1
      }
      if (cq == 0) L.bnd_row[grp] = brow;
      GSTAMP(b0 / BW_RB);
    }
    __syncthreads();
    // combine the cut rows and apply the conv3 ReLU mask; padding rows -> 0
    if (wave >= 2) {
      int br[BW_G];  // the groups' cut rows, read once (three 16-B LDS reads)
#pragma unroll
      for (int g = 0; g < BW_G; g += 4) {
        const int4 t = *reinterpret_cast<const int4*>(&L.bnd_row[g]);
        br[g] = t.x;
        br[g + 1] = t.y;
        br[g + 2] = t.z;
        br[g + 3] = t.w;
      }
#pragma unroll
      for (int u = 0; u < BW_RBG; ++u) {
        const int rr = grp + BW_G * u;
        if (rr >= BW_RB) continue;
        float* d = &L.dz3[rr * SZ3 + 4 * cq];
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (rr < nb) {
          const float2 v01 = *reinterpret_cast<const float2*>(d);
          const float2 v23 = *reinterpret_cast<const float2*>(d + 2);
          v = f32x4{v01.x, v01.y, v23.x, v23.y};
          uint32_t gm = 0;  // groups that continued row rr, added in group order
#pragma unroll
          for (int g = 1; g < BW_G; ++g) gm |= (br[g] == rr ? 1u : 0u) << g;
          while (gm) {
            const int g = __builtin_ctz(gm);
            gm &= gm - 1;
            const f32x4 t = *reinterpret_cast<const f32x4*>(&L.bnd[g][4 * cq]);
            v.x += t.x;
            v.y += t.y;
            v.z += t.z;
            v.w += t.w;
          }
          const uint32_t mk = mask >> (4 * u);
          v.x = (mk & 1u) ? v.x : 0.f;
          v.y = (mk & 2u) ? v.y : 0.f;
          v.z = (mk & 4u) ? v.z : 0.f;
          v.w = (mk & 8u) ? v.w : 0.f;
        }
        *reinterpret_cast<float2*>(d) = make_float2(v.x, v.y);
        *reinterpret_cast<float2*>(d + 2) = make_float2(v.z, v.w);
      }
    }
    __syncthreads();
    BSTAMP(sb_ + 1);

    // ---- c. dX2 = dZ3 W3 (32 x 128 . 128 x 64), 16x16 tile per wave ---------
    {
      f32x4m acc = {0.f, 0.f, 0.f, 0.f};
      if (16 * rt < nb) {
        const float* ap = L.dz3 + (16 * rt + r16) * SZ3 + q;
#pragma unroll
        for (int s = 0; s < 32; ++s)
          acc = mfma16(ap[4 * s], __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(w3r, boff, s * 1024, 0)), acc);
      }
      const int col = 16 * ct + r16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 16 * rt + 4 * q + j;
        L.dz2[row * SZ2 + col] = L.x2[row * S64 + col] > 0.f ? acc[j] : 0.f;
      }
    }
    __syncthreads();
    BSTAMP(sb_ + 2);

    // ---- d. dX1 = dZ2 W2 (32 x 64 . 64 x 64), 16x16 tile per wave -----------
    {
      f32x4m acc = {0.f, 0.f, 0.f, 0.f};
      if (16 * rt < nb) {
        const float* ap = L.dz2 + (16 * rt + r16) * SZ2 + q;
#pragma unroll
        for (int s = 0; s < 16; ++s)
          acc = mfma16(ap[4 * s], __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(w2r, boff, s * 1024, 0)), acc);
      }
      const int col = 16 * ct + r16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 16 * rt + 4 * q + j;
        L.dz1[row * SZ2 + col] = L.x1[row * S64 + col] > 0.f ? acc[j] : 0.f;
      }
    }
    __syncthreads();
    BSTAMP(sb_ + 3);

    // ---- e. weight / bias gradients over the batch rows (32x32x2) ------------
    {
      const int nb2 = (nb + 1) & ~1;
      // dW3[o][i] += sum_rows dz3[row][o] x2[row][i]; wave -> (o tile, i tile)
      const int ot = wave >> 1, it = wave & 1;
      const float* ap = L.dz3 + h * SZ3 + 32 * ot + r32;
      const float* bp = L.x2 + h * S64 + 32 * it + r32;
      for (int s = 0; s < nb2 / 2; ++s) a_dw3 = mfma32(ap[2 * s * SZ3], bp[2 * s * S64], a_dw3);
      // dW2[o][i] += sum_rows dz2[row][o] x1[row][i]; waves 0-3 rows [0,16),
      // waves 4-7 rows [16,32) of the batch, same 4 tiles
      const int t2 = wave & 3, rh = wave >> 2;
      const float* ap2 = L.dz2 + (16 * rh + h) * SZ2 + 32 * (t2 >> 1) + r32;
      const float* bp2 = L.x1 + (16 * rh + h) * S64 + 32 * (t2 & 1) + r32;
      const int n2 = max(0, min(nb2 - 16 * rh, 16)) / 2;
      for (int s = 0; s < n2; ++s) a_dw2 = mfma32(ap2[2 * s * SZ2], bp2[2 * s * S64], a_dw2);
      // rows past nb are zero in dz1 / dz2 / dz3 / pts, so the sums run over all
      // BW_RB rows unrolled (the LDS reads issue together; adding the zeros leaves
      // every partial sum bitwise what the nb-row loop gives)
      if (tid < 192) {
        const int o = tid / 3, i = tid % 3;
#pragma unroll 8
        for (int r = 0; r < BW_RB; ++r) acc_w1 = fmaf(L.dz1[r * SZ2 + o], L.pts[r * 4 + i], acc_w1);
      } else if (tid < 448) {
        const float* src = tid < 320 ? L.dz3 + (tid - 192) : (tid < 384 ? L.dz2 + (tid - 320)
                                                                        : L.dz1 + (tid - 384));
        const int st = tid < 320 ? SZ3 : SZ2;
#pragma unroll 8
        for (int r = 0; r < BW_RB; ++r) acc_b += src[r * st];
      }
    }
    __syncthreads();
    BSTAMP(sb_ + 4);
  }

  // ---- 4. write this workgroup's slab ----------------------------------------
  const int r32 = lane & 31;
  float* slab = slabs + ((size_t)c * gridDim.x + chunk) * SLAB;
  {
    const int ot = wave >> 1, it = wave & 1;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      slab[SL_DW3 + (32 * ot + acc_row(r, lane)) * 64 + 32 * it + r32] = a_dw3[r];
  }
  // the two row halves of dW2 meet in LDS (waves 4-7 park theirs in dz3)
  {
    const int t2 = wave & 3;
    float* pp = L.dz3;
    if (wave >= 4) {
#pragma unroll
      for (int r = 0; r < 16; ++r) pp[t2 * 1024 + r * 64 + lane] = a_dw2[r];
    }
    __syncthreads();
    if (wave < 4) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = a_dw2[r] + pp[t2 * 1024 + r * 64 + lane];
        slab[SL_DW2 + (32 * (t2 >> 1) + acc_row(r, lane)) * 64 + 32 * (t2 & 1) + r32] = v;
      }
    }
  }
  if (tid < 192) slab[SL_DW1 + tid] = acc_w1;
  else if (tid < 320) slab[SL_DB3 + tid - 192] = acc_b;
  else if (tid < 384) slab[SL_DB2 + tid - 320] = acc_b;
  else if (tid < 448) slab[SL_DB1 + tid - 384] = acc_b;
#ifdef PCADV_STAMPS
  __syncthreads();
  if (st_ && threadIdx.x == 0) { st_[14] = __builtin_amdgcn_s_memrealtime(); st_[15] = nact; }
#endif
#undef BSTAMP
#undef GSTAMP
#undef ASTAMP
}

// out[j] = sum over slabs in fixed order: 64 columns per block (one per lane;
// 199 blocks, so with conv4's Adam blocks the launch spreads over most CUs), 16
// waves split the slabs into contiguous ranges, combined in wave order.
constexpr int FIN_COLS = 64;
__device__ void reduce_slabs_block(int blk, float (*part)[64], const float* __restrict__ slabs,
                                   int nslabs, float* dw1, float* db1, float* dw2, float* db2,
                                   float* dw3, float* db3, const FinAdam& fa) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blk * FIN_COLS + lane;
  const int s0 = wave * nslabs / 16, s1 = (wave + 1) * nslabs / 16;
  // Adam state of this lane's parameter, in flight during the reduction
  const bool adam = fa.on && wave == 0 && j < SLAB;
  float ap = 0.f, am = 0.f, av = 0.f;
  if (adam) {
    ap = fa.gp[j];
    am = fa.gm[j];
    av = fa.gv[j];
  }
  // bias corrections (f64 pow) computed while the loads are in flight
  const AdamHp h = adam ? adam_hp(fa.step_count, fa.step_offset, fa.b1, fa.b2, fa.eps, fa.lr_g)
                        : AdamHp{};
  float acc = 0.f;
  if (j < SLAB) {
    // 32 slabs in flight per lane: one round trip per 32 slabs
    int s = s0;
    constexpr int RD = 32;
    for (; s + RD <= s1; s += RD) {
      float v[RD];
#pragma unroll
      for (int u = 0; u < RD; ++u) v[u] = slabs[(size_t)(s + u) * SLAB + j];
#pragma unroll
      for (int u = 0; u < RD; ++u) acc += v[u];
    }
    for (; s + 8 <= s1; s += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slabs[(size_t)(s + u) * SLAB + j];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < s1; ++s) acc += slabs[(size_t)s * SLAB + j];
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && j < SLAB) {
    float x = part[0][lane];
    for (int w = 1; w < 16; ++w) x += part[w][lane];
    if (j < SL_DB1) dw1[j] = x;
    else if (j < SL_DW2) db1[j - SL_DB1] = x;
    else if (j < SL_DB2) dw2[j - SL_DW2] = x;
    else if (j < SL_DW3) db2[j - SL_DB2] = x;
    else if (j < SL_DB3) dw3[j - SL_DW3] = x;
    else db3[j - SL_DB3] = x;
    if (adam) {  // the slab order is the generator's flat order (PCADV_G_CONV1_W = 0 ..)
      adam_elem(ap, x, am, av, h);
      fa.gp[j] = ap;
      fa.gm[j] = am;
      fa.gv[j] = av;
    }
  }
}

// One launch after k_feat_bwd_chunk: FIN_NRED blocks reduce the slabs
// (dW1..db3) and, with the fused Adam, update those parameters; nb4 more
// blocks update conv4's (its gradient came from the chunk launch, whose
// chunks read W4 until they end).  The dW4 gather and the other Adam work rode
// along k_feat_bwd_chunk.
constexpr int FIN_NRED = (SLAB + FIN_COLS - 1) / FIN_COLS;
#ifndef PCADV_FIN_W4_SPREAD
#define PCADV_FIN_W4_SPREAD 1  // A/B builds: 0 = conv4's Adam on the fewest blocks (two float4 per thread)
#endif
constexpr int FIN_W4_V4 = PCADV_FIN_W4_SPREAD ? 1 : 2;
constexpr int FIN_CUS = 256;  // MI355X compute units
__global__ void __launch_bounds__(1024)
k_feat_bwd_finish(const float* __restrict__ slabs, int nslabs, float* dw1, float* db1, float* dw2,
                  float* db2, float* dw3, float* db3, FinAdam fa, int nb4, IterEpi epi) {
  __shared__ float part[16][64];
  const int blk = (int)blockIdx.x;
  // the training iteration's epilogue (pcadv_adv_args.epi_*): the step's
  // losses are final since the launches before this one
  if (blk == 0 && threadIdx.x < 64 && (epi.ncounters > 0 || epi.ring))
    iter_epi_wave(epi, (int)threadIdx.x);
  if (blk < FIN_NRED) {
    reduce_slabs_block(blk, part, slabs, nslabs, dw1, db1, dw2, db2, dw3, db3, fa);
  } else {
    constexpr int64_t W4 = PCADV_G_CONV4_W, N4 = PCADV_G_CONV4_B + PCADV_C4 - PCADV_G_CONV4_W;
    adam_range<1024, FIN_W4_V4>(blk - FIN_NRED, nb4, fa.gp + W4, fa.gm + W4, fa.gv + W4, fa.gg + W4, N4,
                        fa.lr_g, fa);
  }
}

size_t feat_bwd_workspace_bytes(int C, int N) {
  const size_t nchunk = (N + BW_PCH - 1) / BW_PCH;
  return (size_t)C * nchunk * SLAB * sizeof(float);
}

int launch_feat_bwd(const float* dg, const int32_t* gidx, const float* pts_a, const float* pts_b,
                    int split, int C, int N, const float* w1, const float* b1, const float* w2,
                    const float* b2, const float* w3, const float* w4, const float* x3,
                    float* dw1, float* db1, float* dw2, float* db2, float* dw3, float* db3,
                    float* dw4, float* db4, void* ws, size_t ws_bytes, hipStream_t s,
                    uint64_t* stamps, const FinAdam* adam, const int* sortrec,
                    const IterEpi* epi, int x3_bf16) {
  const int O = PCADV_C4;
  PC_REQUIRE(ws_bytes >= feat_bwd_workspace_bytes(C, N), "feat_bwd: workspace too small");
  const int nchunk = (N + BW_PCH - 1) / BW_PCH;
  float* slabs = static_cast<float*>(ws);
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_feat_bwd_chunk<false, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(BwdLds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_feat_bwd_chunk<true, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(BwdLds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_feat_bwd_chunk<false, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(BwdLds)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_feat_bwd_chunk<true, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(BwdLds)) != hipSuccess) {
      set_error("feat_bwd: cannot reserve %zu bytes of LDS", sizeof(BwdLds));
      return PCADV_EHIP;
    }
    attr_set = true;
  }
  PC_REQUIRE(dw4 && db4, "feat_bwd: dw4/db4 required");
  FinAdam fa{};
  int nba0 = 0, nba1 = 0;  // Adam workgroups (BW_T threads) of the chunk launch
  if (adam && adam->on) {
    fa = *adam;
    PC_REQUIRE(fa.gp && fa.gm && fa.gv && fa.gg && fa.step_count && fa.g_n > fa.g_rest0 &&
                   fa.g_rest0 % 4 == 0 && (fa.d_n == 0 || (fa.dp && fa.dm && fa.dv && fa.dg)) &&
                   dw1 == fa.gg + PCADV_G_CONV1_W && dw4 == fa.gg + PCADV_G_CONV4_W &&
                   db4 == fa.gg + PCADV_G_CONV4_B,
               "feat_bwd: the fused Adam needs the generator's flat buffers");
    nba0 = fin_adam_blocks(fa.g_n - fa.g_rest0, BW_T, FIN_ADAM_V4);
    nba1 = fa.d_n > 0 ? fin_adam_blocks(fa.d_n, BW_T, FIN_ADAM_V4) : 0;
  }
  // trailing workgroup rows: the dW4 gather (NDW4), then the Adam workgroups
  PC_REQUIRE(O == BW_MAXO, "feat_bwd: %d pooled channels (expects %d)", O, BW_MAXO);
  constexpr int NDW4 = BW_MAXO / (BW_T / 64 / DW4_WPC);
  const int arows = (NDW4 + nba0 + nba1 + nchunk - 1) / nchunk;
  auto kern = sortrec ? (x3_bf16 ? k_feat_bwd_chunk<true, true> : k_feat_bwd_chunk<true, false>)
                      : (x3_bf16 ? k_feat_bwd_chunk<false, true> : k_feat_bwd_chunk<false, false>);
  hipLaunchKernelGGL(kern, dim3(nchunk, C + arows), dim3(BW_T), sizeof(BwdLds), s, dg, gidx, O,
                     pts_a, pts_b, split, N, w1, b1, w2, b2, w3, w4, x3, slabs, stamps, sortrec, C,
                     dw4, db4, fa, nba0, nba1);
  PC_HIP_CHECK_LAUNCH("k_feat_bwd_chunk");
  // conv4's Adam spread over the CUs the slab reduction leaves free (one
  // float4 per thread), so no workgroup moves more than a reduction block does
  int nb4 = 0;
  if (fa.on) {
    nb4 = fin_adam_blocks(PCADV_G_CONV4_B + PCADV_C4 - PCADV_G_CONV4_W, 1024, FIN_W4_V4);
    if (PCADV_FIN_W4_SPREAD && nb4 < FIN_CUS - FIN_NRED) nb4 = FIN_CUS - FIN_NRED;
  }
  hipLaunchKernelGGL(k_feat_bwd_finish, dim3(FIN_NRED + nb4), dim3(1024), 0, s, slabs, C * nchunk,
                     dw1, db1, dw2, db2, dw3, db3, fa, nb4, epi ? *epi : IterEpi{});
  PC_HIP_CHECK_LAUNCH("k_feat_bwd_finish");
  return PCADV_OK;
}

}  // namespace pcadv

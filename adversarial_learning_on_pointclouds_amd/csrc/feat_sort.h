// The hit sort of the sparse max-pool backward (feat_bwd.hip, phases 1-3 of
// k_feat_bwd_chunk), as a standalone step that needs only the pooled argmax
// (gidx) and no gradient: the adversarial step runs it early, in workgroups
// that ride along the discriminator tail's launch (tail.hip), and the chunk
// kernel then loads the result instead of sorting on its critical path.
//
// Per (cloud c, 128-point chunk): the channels o whose argmax gidx[c][o] falls
// in the chunk ("hits"), grouped by row (point) in increasing row order and by
// o inside a row; the active rows (rows with hits) in increasing order, and
// the first hit of each.  Record layout (ints, FS_REC per chunk):
//   [0] nact, [1] nhits, [FSR_ROWS + s] row of active slot s (s < nact),
//   [FSR_HOFF + s] first hit of slot s (s <= nact; [nact] = nhits),
//   [FSR_SO + j] o of hit j (j < nhits).
#pragma once
#include "common.h"

namespace pcadv {

constexpr int FS_PCH = 128;    // points per chunk (k_feat_bwd_chunk's BW_PCH)
constexpr int FS_MAXO = 1024;  // channels of the pooled layer
constexpr int FS_T = 512;      // threads per chunk
constexpr int FSR_ROWS = 4, FSR_HOFF = FSR_ROWS + FS_PCH, FSR_SO = FSR_HOFF + FS_PCH + 4;
constexpr int FS_REC = FSR_SO + FS_MAXO;

struct SortLds {
  int rcnt[FS_PCH];   // hits per row
  int fill[FS_PCH];   // placement cursor per row
  int roff[FS_PCH];   // first hit of each row
  int key[FS_MAXO];   // o of each hit, grouped by row (arbitrary order in a row)
  int wsum[2], wact[2];
};

// One chunk on FS_T threads (t = 0 .. FS_T - 1, every thread of the workgroup
// reaches the same barriers; valid = false: barriers only).  gidx_c: the
// cloud's argmax row [O]; p0: the chunk's first point.
__device__ __forceinline__ void chunk_sort(const int32_t* __restrict__ gidx_c, int O, int p0, int t,
                                           bool valid, SortLds& L, int* __restrict__ rec) {
  const int lane = t & 63, wave = t >> 6;
  int ga[2];  // the argmax rows, loaded before the counters are cleared
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int o = u * FS_T + t;
    ga[u] = valid && o < O ? gidx_c[o] : -1;
  }
  if (t < FS_PCH) {
    L.rcnt[t] = 0;
    L.fill[t] = 0;
  }
  __syncthreads();
  int hrow[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int a = ga[u];
    const bool hit = a >= p0 && a < p0 + FS_PCH;
    hrow[u] = hit ? a - p0 : -1;
    if (hit) atomicAdd(&L.rcnt[a - p0], 1);
  }
  __syncthreads();
  // active rows compacted in row order; row offsets = exclusive scan of counts
  if (wave < 2) {
    const int cnt = L.rcnt[t];
    int v = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int x = __shfl_up(v, d);
      if (lane >= d) v += x;
    }
    const uint64_t m = __ballot(cnt > 0);
    if (lane == 63) {
      L.wsum[wave] = v;
      L.wact[wave] = __popcll(m);
    }
    L.roff[t] = v - cnt;
  }
  __syncthreads();
  if (wave < 2) {
    const int cnt = L.rcnt[t];
    const uint64_t m = __ballot(cnt > 0);
    const int slot = (wave ? L.wact[0] : 0) + __popcll(m & ((1ull << lane) - 1ull));
    const int off = L.roff[t] + (wave ? L.wsum[0] : 0);
    L.roff[t] = off;
    if (valid && cnt > 0) {
      rec[FSR_ROWS + slot] = t;
      rec[FSR_HOFF + slot] = off;
    }
    if (valid && t == 0) {
      const int nact = L.wact[0] + L.wact[1], nhits = L.wsum[0] + L.wsum[1];
      rec[0] = nact;
      rec[1] = nhits;
      rec[FSR_HOFF + nact] = nhits;
    }
  }
  __syncthreads();
  // place each hit in its row's segment, then rank it there by o
  int hpos[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    hpos[u] = -1;
    if (hrow[u] >= 0) {
      hpos[u] = L.roff[hrow[u]] + atomicAdd(&L.fill[hrow[u]], 1);
      L.key[hpos[u]] = u * FS_T + t;
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (hrow[u] >= 0) {
      const int o = u * FS_T + t, s0 = L.roff[hrow[u]], s1 = s0 + L.rcnt[hrow[u]];
      int rank = 0;
      for (int j = s0; j < s1; ++j) rank += L.key[j] < o;
      rec[FSR_SO + s0 + rank] = o;
    }
  }
}

}  // namespace pcadv

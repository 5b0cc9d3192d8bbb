// PointNetfeat backward on gfx950: autograd of models/pointnet.py:115-130.
//
// The max-pool has no ReLU before it (pointnet.py:128-129), so channel o of
// cloud c sends its whole gradient to the single point gidx[c][o]:
//   dW4[o,:] = sum_c g[c,o] x3[c, gidx[c,o], :]            (k_dw4_gather)
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
// k_reduce_slabs sums the slabs in a fixed order (no atomics).
#include "common.h"

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

struct BwdLds {
  int key[BW_MAXO];          // (row << 10) | o of each hit, generation order
  float hg[BW_MAXO];         // g of each hit, generation order
  int so[BW_MAXO];           // sorted o
  float sg[BW_MAXO];         // sorted g
  int wcnt[8], wact[8];
  int slot_of_row[BW_PCH];   // active flag, then compact slot (-1 if inactive)
  int rows_list[BW_PCH];     // compact slot -> row
  int hoff[BW_PCH + 4];      // first sorted hit of each compact slot
  alignas(16) float dz3[BW_RB * SZ3];
  alignas(16) float x2[BW_RB * S64];   // recomputed conv2 output (f32, as the forward)
  alignas(16) float x1[BW_RB * S64];   // recomputed conv1 output
  alignas(16) float dz2[BW_RB * SZ2];
  alignas(16) float dz1[BW_RB * SZ2];
  alignas(16) float pts[BW_RB * 4];
};

__global__ void __launch_bounds__(BW_T, 4)
k_feat_bwd_chunk(const float* __restrict__ dg, const int32_t* __restrict__ gidx, int O,
                 const float* __restrict__ pts_a, const float* __restrict__ pts_b, int split,
                 int N, const float* __restrict__ w1, const float* __restrict__ b1,
                 const float* __restrict__ w2, const float* __restrict__ b2,
                 const float* __restrict__ w3, const float* __restrict__ w4,
                 const float* __restrict__ x3, float* __restrict__ slabs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  BwdLds& L = *reinterpret_cast<BwdLds*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5, r16 = lane & 15, q = lane >> 4;
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
  const int boff = (q * 64 + 16 * ct + r16) * 4;
  if (tid < BW_PCH) L.slot_of_row[tid] = 0;
  __syncthreads();

  // ---- 1a. hits in increasing o (wave w scans channels [w*O/8, (w+1)*O/8)) ----
  const int per_wave = O / 8;
  {
    int cnt = 0;
    for (int base = 0; base < per_wave; base += 64) {
      const int o = wave * per_wave + base + lane;
      const int a = gidx[(size_t)c * O + o];
      const bool hit = a >= p0 && a < p0 + BW_PCH;
      const uint64_t m = __ballot(hit);
      if (hit) {
        const int pos = wave * per_wave + cnt + __popcll(m & ((1ull << lane) - 1ull));
        L.key[pos] = ((a - p0) << 10) | o;
        L.hg[pos] = dg[(size_t)c * O + o];
        L.slot_of_row[a - p0] = 1;
      }
      cnt += __popcll(m);
    }
    if (lane == 0) L.wcnt[wave] = cnt;
  }
  __syncthreads();

  // ---- 2. compact the active rows (threads 0..127 own one row each) ----------
  int nact = 0, nhits = 0;
  {
    const bool f = tid < BW_PCH && L.slot_of_row[tid] != 0;
    const uint64_t m = __ballot(f);
    if (lane == 0) L.wact[wave] = __popcll(m);
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wave; ++w) off += L.wact[w];
    for (int w = 0; w < 8; ++w) {
      nact += L.wact[w];
      nhits += L.wcnt[w];
    }
    const int slot = off + __popcll(m & ((1ull << lane) - 1ull));
    if (tid < BW_PCH) L.slot_of_row[tid] = f ? slot : -1;
    if (f) L.rows_list[slot] = tid;
  }
  __syncthreads();

  // ---- 1b. rank-count sort of the hits by key = (row, o) ---------------------
  auto phys = [&](int j) {
    int w = 0;
    while (w < 7 && j >= L.wcnt[w]) { j -= L.wcnt[w]; ++w; }
    return w * per_wave + j;
  };
  for (int j = tid; j < nhits; j += BW_T) {
    const int pj = phys(j);
    const int kj = L.key[pj];
    int rank = 0;
    for (int w = 0; w < 8; ++w) {
      const int n = L.wcnt[w];
      const int* kp = &L.key[w * per_wave];
      for (int i = 0; i < n; ++i) rank += kp[i] < kj;
    }
    L.so[rank] = kj & 1023;
    L.sg[rank] = L.hg[pj];
  }
  {
    // hits per compact slot (one thread per slot), inclusive scan -> hoff
    int cnt = 0;
    if (tid < nact) {
      const int row = L.rows_list[tid];
      for (int w = 0; w < 8; ++w) {
        const int n = L.wcnt[w];
        const int* kp = &L.key[w * per_wave];
        for (int i = 0; i < n; ++i) cnt += (kp[i] >> 10) == row;
      }
    }
    int v = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(v, d);
      if (lane >= d) v += t;
    }
    __syncthreads();  // wact reads of step 2 are done
    if (lane == 63) L.wact[wave] = v;
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wave; ++w) off += L.wact[w];
    if (tid < BW_PCH) L.hoff[tid + 1] = off + v;
    if (tid == 0) L.hoff[0] = 0;
  }
  __syncthreads();

  // register accumulators that live across batches
  f32x16 a_dw3 = {}, a_dw2 = {};
  float acc_w1 = 0.f, acc_b = 0.f;

  for (int b0 = 0; b0 < nact; b0 += BW_RB) {
    const int nb = min(BW_RB, nact - b0);
    // ---- a. recompute x1, x2 of the batch rows from their points, with the
    //      forward's exact operation order (bit-identical activations) --------
    if (tid < BW_RB * 3) {
      const int r = tid / 3, k = tid % 3;
      L.pts[r * 4 + k] = r < nb ? pts[(size_t)(p0 + L.rows_list[b0 + r]) * 3 + k] : 0.f;
    }
    __syncthreads();
    {
      const int ch = tid & 63, rg = tid >> 6;  // 8 groups x 4 rows
      const float wa = w1[ch * 3 + 0], wb = w1[ch * 3 + 1], wc = w1[ch * 3 + 2], bb = b1[ch];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rr = 4 * rg + u;
        L.x1[rr * S64 + ch] = conv1_point(wa, wb, wc, bb, L.pts[rr * 4 + 0], L.pts[rr * 4 + 1],
                                          L.pts[rr * 4 + 2]);
      }
    }
    __syncthreads();
    if (wave < 2) {
      f32x4 bf[8];
      load_bfrag<64>(w2, 32 * wave, lane, bf);
      f32x16 acc = {};
      acc = mfma_rows_x_wt<64>(L.x1, S64, bf, acc, lane);
      const int col = 32 * wave + r32;
      const float bias = b2[col];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = acc[i] + bias;
        L.x2[acc_row(i, lane) * S64 + col] = v > 0.f ? v : 0.f;
      }
    }

    // ---- b. dZ3 rows: thread = (column i, 8-row group); the hits of a
    //      contiguous row range are contiguous in the sorted list -------------
    {
      const int i = tid & 127, rg = tid >> 7;
      const int s0 = b0 + 8 * rg, s1 = min(s0 + 8, b0 + nb);
      uint32_t mask = 0;  // conv3 ReLU mask of my rows, prefetched
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int s = s0 + u;
        if (s < s1) {
          const size_t p = (size_t)c * N + p0 + L.rows_list[s];
          mask |= (x3[p * 128 + i] > 0.f ? 1u : 0u) << u;
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) L.dz3[(8 * rg + u) * SZ3 + i] = 0.f;
      if (s0 < s1) {
        int s = s0;
        const int j1 = L.hoff[s1];
        int jnext = L.hoff[s + 1];
        float acc = 0.f;
        int j = L.hoff[s0];
        auto flush = [&]() {
          L.dz3[(s - b0) * SZ3 + i] = ((mask >> (s - s0)) & 1u) ? acc : 0.f;
          acc = 0.f;
          ++s;
          jnext = L.hoff[s + 1];
        };
        for (; j + 8 <= j1; j += 8) {
          float wv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) wv[u] = w4[(size_t)L.so[j + u] * 128 + i];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            while (j + u >= jnext) flush();
            acc = fmaf(L.sg[j + u], wv[u], acc);
          }
        }
        for (; j + 4 <= j1; j += 4) {
          float wv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) wv[u] = w4[(size_t)L.so[j + u] * 128 + i];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            while (j + u >= jnext) flush();
            acc = fmaf(L.sg[j + u], wv[u], acc);
          }
        }
        for (; j < j1; ++j) {
          const float wv = w4[(size_t)L.so[j] * 128 + i];
          while (j >= jnext) flush();
          acc = fmaf(L.sg[j], wv, acc);
        }
        flush();  // every active row has at least one hit: s ends at s1
      }
    }
    __syncthreads();

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
      if (tid < 192) {
        const int o = tid / 3, i = tid % 3;
        for (int r = 0; r < nb; ++r) acc_w1 = fmaf(L.dz1[r * SZ2 + o], L.pts[r * 4 + i], acc_w1);
      } else if (tid < 320) {
        for (int r = 0; r < nb; ++r) acc_b += L.dz3[r * SZ3 + tid - 192];
      } else if (tid < 384) {
        for (int r = 0; r < nb; ++r) acc_b += L.dz2[r * SZ2 + tid - 320];
      } else if (tid < 448) {
        for (int r = 0; r < nb; ++r) acc_b += L.dz1[r * SZ2 + tid - 384];
      }
    }
    __syncthreads();
  }

  // ---- 4. write this workgroup's slab ----------------------------------------
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
}

// out[j] = sum over slabs in fixed order: 128 columns per block (lanes hold
// float2), 16 waves split the slabs into contiguous ranges, combined in wave
// order through LDS.
__global__ void __launch_bounds__(1024)
k_reduce_slabs(const float* __restrict__ slabs, int nslabs, float* dw1, float* db1, float* dw2,
               float* db2, float* dw3, float* db3) {
  __shared__ float2 part[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * 128 + 2 * lane;  // SLAB is even: j, j+1 both valid or both not
  const int s0 = wave * nslabs / 16, s1 = (wave + 1) * nslabs / 16;
  float2 acc = make_float2(0.f, 0.f);
  if (j < SLAB) {
    int s = s0;
    for (; s + 8 <= s1; s += 8) {
      float2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float2*>(slabs + (size_t)(s + u) * SLAB + j);
#pragma unroll
      for (int u = 0; u < 8; ++u) { acc.x += v[u].x; acc.y += v[u].y; }
    }
    for (; s < s1; ++s) {
      const float2 v = *reinterpret_cast<const float2*>(slabs + (size_t)s * SLAB + j);
      acc.x += v.x;
      acc.y += v.y;
    }
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && j < SLAB) {
    float2 v = part[0][lane];
    for (int w = 1; w < 16; ++w) { v.x += part[w][lane].x; v.y += part[w][lane].y; }
    const float vv[2] = {v.x, v.y};
    for (int e = 0; e < 2; ++e) {
      const int jj = j + e;
      const float x = vv[e];
      if (jj < SL_DB1) dw1[jj] = x;
      else if (jj < SL_DW2) db1[jj - SL_DB1] = x;
      else if (jj < SL_DB2) dw2[jj - SL_DW2] = x;
      else if (jj < SL_DW3) db2[jj - SL_DB2] = x;
      else if (jj < SL_DB3) dw3[jj - SL_DW3] = x;
      else db3[jj - SL_DB3] = x;
    }
  }
}

// dW4[o,:] = sum_c g[c,o] x3[c, gidx[c,o], :];  db4[o] = sum_c g[c,o].
// One wave per channel, lanes hold two of the 128 columns.
__global__ void __launch_bounds__(256)
k_dw4_gather(const float* __restrict__ dg, const int32_t* __restrict__ gidx, int C, int N, int O,
             const float* __restrict__ x3, float* __restrict__ dw4, float* __restrict__ db4) {
  const int lane = threadIdx.x & 63;
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= O) return;
  float ax = 0.f, ay = 0.f, ab = 0.f;
  int c = 0;
  for (; c + 8 <= C; c += 8) {
    float g[8];
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      g[u] = dg[(size_t)(c + u) * O + o];
      const int n = gidx[(size_t)(c + u) * O + o];
      v[u] = *reinterpret_cast<const float2*>(x3 + ((size_t)(c + u) * N + n) * 128 + 2 * lane);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ax = fmaf(g[u], v[u].x, ax);
      ay = fmaf(g[u], v[u].y, ay);
      ab += g[u];
    }
  }
  for (; c < C; ++c) {
    const float g = dg[(size_t)c * O + o];
    const int n = gidx[(size_t)c * O + o];
    const float2 v = *reinterpret_cast<const float2*>(x3 + ((size_t)c * N + n) * 128 + 2 * lane);
    ax = fmaf(g, v.x, ax);
    ay = fmaf(g, v.y, ay);
    ab += g;
  }
  *reinterpret_cast<float2*>(dw4 + (size_t)o * 128 + 2 * lane) = make_float2(ax, ay);
  if (lane == 0) db4[o] = ab;
}

size_t feat_bwd_workspace_bytes(int C, int N) {
  const size_t nchunk = (N + BW_PCH - 1) / BW_PCH;
  return (size_t)C * nchunk * SLAB * sizeof(float);
}

int launch_dw4_gather(const float* dg, const int32_t* gidx, int C, int N, const float* x3,
                      float* dw4, float* db4, hipStream_t s);

int launch_feat_bwd(const float* dg, const int32_t* gidx, const float* pts_a, const float* pts_b,
                    int split, int C, int N, const float* w1, const float* b1, const float* w2,
                    const float* b2, const float* w3, const float* w4, const float* x3,
                    float* dw1, float* db1, float* dw2, float* db2, float* dw3, float* db3,
                    float* dw4, float* db4, void* ws, size_t ws_bytes, hipStream_t s) {
  const int O = PCADV_C4;
  PC_REQUIRE(ws_bytes >= feat_bwd_workspace_bytes(C, N), "feat_bwd: workspace too small");
  const int nchunk = (N + BW_PCH - 1) / BW_PCH;
  float* slabs = static_cast<float*>(ws);
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_feat_bwd_chunk),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(BwdLds)) != hipSuccess) {
      set_error("feat_bwd: cannot reserve %zu bytes of LDS", sizeof(BwdLds));
      return PCADV_EHIP;
    }
    attr_set = true;
  }
  hipLaunchKernelGGL(k_feat_bwd_chunk, dim3(nchunk, C), dim3(BW_T), sizeof(BwdLds), s, dg, gidx, O,
                     pts_a, pts_b, split, N, w1, b1, w2, b2, w3, w4, x3, slabs);
  PC_HIP_CHECK_LAUNCH("k_feat_bwd_chunk");
  hipLaunchKernelGGL(k_reduce_slabs, dim3((SLAB + 127) / 128), dim3(1024), 0, s, slabs, C * nchunk,
                     dw1, db1, dw2, db2, dw3, db3);
  PC_HIP_CHECK_LAUNCH("k_reduce_slabs");
  if (dw4) return launch_dw4_gather(dg, gidx, C, N, x3, dw4, db4, s);
  return PCADV_OK;
}

// dW4 / db4 alone (independent of k_feat_bwd_chunk: the fused step runs it on
// a second stream)
int launch_dw4_gather(const float* dg, const int32_t* gidx, int C, int N, const float* x3,
                      float* dw4, float* db4, hipStream_t s) {
  const int O = PCADV_C4;
  hipLaunchKernelGGL(k_dw4_gather, dim3((O + 3) / 4), dim3(256), 0, s, dg, gidx, C, N, O, x3,
                     dw4, db4);
  PC_HIP_CHECK_LAUNCH("k_dw4_gather");
  return PCADV_OK;
}

}  // namespace pcadv

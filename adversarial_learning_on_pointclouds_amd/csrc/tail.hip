// Row-block fused kernels for the small end of the adversarial step (gfx950).
//
// At B = 32 every layer of the classifier head and of the discriminator is a
// few hundred kFLOP, so a launch per layer costs more than the layer.  Where a
// chain of layers has small weights, one workgroup takes 16 rows through the
// whole chain with the activations in LDS:
//
//   k_head_fwd  fc3 (models/pointnet.py:202) -> log_softmax / CrossEntropy
//               (utils/trainer.py:469-472,492) -> discriminator conv1 + LeakyReLU
//               (models/discriminator.py:43) for the GT and noGT rows
//   k_disc_tail discriminator conv4 -> conv5 -> fc (discriminator.py:46-51), the
//               BCE terms of trainer.py:507,537,553 with make_D_label's soft
//               labels (utils/utils.py:22-31), then back through fc, conv5 and
//               conv4 to dL/d(conv3 output); per-workgroup partial weight
//               gradients of conv4/conv5/fc (summed by a later launch)
//   k_head_bwd  discriminator conv1 input gradient of the adversarial rows ->
//               log_softmax backward -> fc3 input gradient; extra workgroups
//               compute conv1's weight gradient; finalises the four losses
//
// Each layer is a set of 16x16 output tiles on v_mfma_f32_16x16x4_f32 (exact
// f32), one reduction chunk of <= 128 per work item; items are spread over the
// 16 waves and their partial tiles summed in a fixed order.
#include "common.h"
#include "feat_sort.h"

namespace pcadv {

constexpr int TR = 16;     // rows per workgroup
constexpr int TT = 1024;   // 16 waves

struct SemiArgs {           // run_training_semi's pseudo-label term (k_head_bwd)
  int on;
  float lambda, th;
  const float* logits;      // [2B][40] generator logits (no-GT rows [B, 2B))
  const float* dout;        // [3B] D logits (adversarial rows [2B, 3B))
};
constexpr int TW = TT / 64;

typedef float f32x4t __attribute__((ext_vector_type(4)));

#ifdef PCADV_STAMPS
// diagnostic build only: phase timestamps (s_memrealtime) [kernel][block][16]
__device__ uint64_t g_tail_stamps[3][16][16];
#define TSTAMP(kern, k) do { if (threadIdx.x == 0 && blockIdx.x < 16) g_tail_stamps[kern][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define TSTAMP(kern, k) do { } while (0)
#endif
__device__ __forceinline__ f32x4t mfma16t(float a, float b, f32x4t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

enum BMode { B_OK = 0, B_KO = 1 };  // B[k][j] = W[j * ldw + k]  |  W[k * ldw + j]

// out[r][j] = act(sum_k A[r][k] B[k][j] + bias[j]) for the 16 rows, j < NC.
// A: LDS [16][as]; W: weights in LDS (staged by lds_fill) or global; out: LDS
// or global [16][os].  One work item = one 16x16 output tile over a reduction
// chunk of <= 128; with a single chunk the tile goes straight to `out`,
// otherwise the chunk partials meet in scratch (>= items * 256 floats, LDS).
// Rows >= dup_row are also written at out + dup_off (the duplicated noGT rows
// of the discriminator input).
// KC0: reduction chunk per work item (default min(K, 128)); smaller chunks
// spread a narrow layer over more waves at the cost of a partial-sum pass.
// Output mask (backward layers): with `om`, each output is multiplied by
// act'(om[row][j]) for OM_ACT, then by om_drop[row][j] * om_keep when given, so
// it is stored as the next backward layer's dz.
struct OutMask {
  const float* om;      // [rows][oms] activations of the layer below (LDS or global)
  int oms;
  const float* drop;    // [rows][oms] {0,1} dropout mask or nullptr
  float keep;
};
template <int K, int NC, int MODE, int ACT, int KC0 = 128, int OM_ACT = ACT_NONE>
__device__ __forceinline__ void rows_layer(const float* A, int as, const float* W, int ldw,
                                           const float* __restrict__ bias, float* out, int os,
                                           float* scratch, int nrows = TR, int dup_row = TR,
                                           long dup_off = 0, OutMask msk = OutMask{}) {
  auto masked = [&](float o, int row, int j) {
    if (OM_ACT != ACT_NONE) o *= act_bwd(msk.om[row * msk.oms + j], OM_ACT);
    if (msk.drop) o *= msk.drop[row * msk.oms + j] * msk.keep;
    return o;
  };
  constexpr int KC = K < KC0 ? K : KC0;
  constexpr int C = (K + KC - 1) / KC, T = (NC + 15) / 16, ITEMS = T * C;
  constexpr int NS = (KC + 3) / 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, q = lane >> 4;
  for (int it = wave; it < ITEMS; it += TW) {
    const int t = it / C, c = it % C, j = 16 * t + r, k0 = c * KC;
    // every operand read is issued before the first MFMA of the tile
    float av[NS], bv[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k = k0 + 4 * s + q;
      const bool vk = k < K && 4 * s + q < KC, v = vk && j < NC;
      const int jj = v ? j : 0, kk = v ? k : 0;
      const float w = MODE == B_OK ? W[jj * ldw + kk] : W[kk * ldw + jj];
      const float a = A[r * as + (vk ? k : 0)];
      bv[s] = v ? w : 0.f;
      av[s] = vk ? a : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMA chain
    f32x4t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) acc = mfma16t(av[s], bv[s], acc);
    if (C == 1) {
      if (j < NC) {
        const float bj = bias ? bias[j] : 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = 4 * q + v;
          if (row < nrows) {
            const float o = masked(act_fwd(acc[v] + bj, ACT), row, j);
            out[row * os + j] = o;
            if (row >= dup_row) out[row * os + j + dup_off] = o;
          }
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v) scratch[it * 256 + (4 * q + v) * 16 + r] = acc[v];
    }
  }
  __syncthreads();
  if (C > 1) {
    for (int e = tid; e < nrows * NC; e += TT) {
      const int row = e / NC, col = e % NC, t = col >> 4;
      float v = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) v += scratch[(t * C + c) * 256 + row * 16 + (col & 15)];
      if (bias) v += bias[col];
      const float o = masked(act_fwd(v, ACT), row, col);
      out[row * os + col] = o;
      if (row >= dup_row) out[row * os + col + dup_off] = o;
    }
    __syncthreads();
  }
}

// Staging of global row-major matrices into LDS (padded row stride `ld`,
// cols % 4 == 0; rows past `valid` are zero-filled).  All the float4 loads of
// a thread (<= 8) are issued before any LDS store: one memory round trip for
// every matrix of the kernel.  No barrier (the caller syncs).
struct Fill {
  float* dst;
  int ld;
  const float* src;
  int rows, cols, valid;
};

__device__ f32x4 kFillZero = {0.f, 0.f, 0.f, 0.f};  // global (not constant): global_load

// FLAT (default): one unconditional load per piece, from a selected address
// (zeros past the matrices and their valid rows).  A load inside a branch made
// the compiler wait for it at the branch's end, one memory round trip per
// piece (k_head_fwd 7.36 -> 6.40 us, A/B); k_cls_head measured 0.3 us slower
// flat and keeps the branches.
template <int NF, int NPT = 8, bool FLAT = true>
__device__ __forceinline__ void lds_fill(const Fill (&f)[NF]) {
  int base[NF + 1];
  base[0] = 0;
#pragma unroll
  for (int d = 0; d < NF; ++d) base[d + 1] = base[d] + f[d].rows * (f[d].cols / 4);
  f32x4 v[NPT];
  if constexpr (FLAT) {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int e = threadIdx.x + u * TT;
      const float* src = reinterpret_cast<const float*>(&kFillZero);
#pragma unroll
      for (int d = 0; d < NF; ++d) {
        const int c4 = f[d].cols / 4, row = (e - base[d]) / c4, col = (e - base[d]) % c4;
        src = e >= base[d] && e < base[d + 1] && row < f[d].valid
                  ? f[d].src + (size_t)row * f[d].cols + 4 * col : src;
      }
      v[u] = *reinterpret_cast<const f32x4*>(src);
    }
  } else {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int e = threadIdx.x + u * TT;
      v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int d = 0; d < NF; ++d)
        if (e >= base[d] && e < base[d + 1]) {
          const int c4 = f[d].cols / 4, row = (e - base[d]) / c4, col = (e - base[d]) % c4;
          if (row < f[d].valid)
            v[u] = *reinterpret_cast<const f32x4*>(f[d].src + (size_t)row * f[d].cols + 4 * col);
        }
    }
  }
#pragma unroll
  for (int u = 0; u < NPT; ++u) {
    const int e = threadIdx.x + u * TT;
#pragma unroll
    for (int d = 0; d < NF; ++d)
      if (e >= base[d] && e < base[d + 1]) {
        const int c4 = f[d].cols / 4, row = (e - base[d]) / c4, col = (e - base[d]) % c4;
        float* p = f[d].dst + row * f[d].ld + 4 * col;
        p[0] = v[u][0];
        p[1] = v[u][1];
        p[2] = v[u][2];
        p[3] = v[u][3];
      }
  }
}

// ---------------------------------------------------------------------------
// k_head_fwd: rows m of the 2B generator outputs
// ---------------------------------------------------------------------------
// The discriminator conv1 outputs (512 columns) are split over HF_SPLIT
// workgroups per row block; each recomputes fc3 and log_softmax of its 16 rows
// (a fifth of the conv1 work), and split 0 alone writes the head's outputs.
constexpr int HF_SPLIT = 4;
constexpr int HF_COLS = 512 / HF_SPLIT;
struct HeadFwdLds {
  float w1[HF_COLS * 44];      // this split's rows of the D conv1 weight [512][40], padded
  float w3[40 * 260];          // fc3 weight [40][256], padded rows
  float b1[HF_COLS];
  float b3[40];
  alignas(16) float h2[TR * 260];
  float lg[TR * 44];
  float lsm[TR * 44];
  float rl[TR];
  alignas(16) float scratch[12 * 256];
};

__global__ void __launch_bounds__(TT)
k_head_fwd(const float* __restrict__ h2, const float* __restrict__ w3, const float* __restrict__ b3,
           const int64_t* __restrict__ labels, int B, float lambda_cls, float* __restrict__ logits,
           float* __restrict__ dlogits, float* __restrict__ din, const float* __restrict__ dw1,
           const float* __restrict__ db1, float* __restrict__ d1, float* __restrict__ lpart) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  HeadFwdLds& L = *reinterpret_cast<HeadFwdLds*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  TSTAMP(0, 0);
  kernarg_prefetch(h2, w3, b3, labels, B, lambda_cls, logits, dlogits, din, dw1, db1, d1, lpart);
  const int rb = blockIdx.x / HF_SPLIT, sp = blockIdx.x % HF_SPLIT, j0 = sp * HF_COLS;
  const int C = 2 * B, r0 = rb * TR, nrows = min(TR, C - r0);
  const int label = wave < nrows && r0 + wave < B ? (int)labels[r0 + wave] : 0;
  {
    const Fill f[5] = {{L.w1, 44, dw1 + (size_t)j0 * 40, HF_COLS, 40, HF_COLS},
                       {L.h2, 260, h2 + (size_t)r0 * 256, TR, 256, nrows},
                       {L.b1, HF_COLS, db1 + j0, 1, HF_COLS, 1}, {L.b3, 40, b3, 1, 40, 1},
                       {L.w3, 260, w3, 40, 256, 40}};
    lds_fill<5, 5>(f);  // 4362 float4: <= 5 per thread
  }
  __syncthreads();
  TSTAMP(0, 1);
  // reduction chunks of 64: twelve 16-MFMA chains instead of six of 32
  rows_layer<256, 40, B_OK, ACT_NONE, 64>(L.h2, 260, L.w3, 260, L.b3, L.lg, 44, L.scratch);
  TSTAMP(0, 2);
  // log_softmax, CrossEntropy (GT rows), discriminator input rows: one wave per row
  {
    const int row = wave, m = r0 + row;
    const float v = lane < 40 ? L.lg[row * 44 + lane] : -INFINITY;
    float mx = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    const float e = lane < 40 ? expf(v - mx) : 0.f;
    float se = e;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const float lsm = (v - mx) - logf(se);
    if (lane < 40) L.lsm[row * 44 + lane] = lsm;
    float rloss = 0.f;
    if (sp == 0 && m < C && lane < 40) {
      logits[(size_t)m * 40 + lane] = v;
      din[(size_t)m * 40 + lane] = lsm;
      if (m >= B) din[(size_t)(m + B) * 40 + lane] = lsm;
    }
    if (sp == 0 && m < B) {
      const int y = label;
      const float sm = expf(lsm);
      if (lane < 40)
        dlogits[(size_t)m * 40 + lane] = lambda_cls * ((lane == y ? sm - 1.f : sm) / (float)B);
      rloss = -__shfl(lsm, y);
    }
    if (lane == 0) L.rl[row] = rloss;
  }
  __syncthreads();
  if (sp == 0 && wave == 0) {  // the block's CE sum: a fixed butterfly over wave 0
    float s = lane < TR ? L.rl[lane] : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) lpart[rb] = s;
  }
  // D conv1 on the GT rows (D rows [0,B)) and noGT rows (D rows [B,2B) and,
  // identical, [2B,3B)): rows r0.. of d1, copied to r0+B.. for noGT blocks
  TSTAMP(0, 3);
  rows_layer<40, HF_COLS, B_OK, ACT_LRELU>(L.lsm, 44, L.w1, 44, L.b1,
                                           d1 + (size_t)r0 * 512 + j0, 512, nullptr, nrows,
                                           max(0, B - r0), (long)B * 512);
  TSTAMP(0, 4);
}

// ---------------------------------------------------------------------------
// k_disc_tail: rows m of the 3B discriminator rows
// ---------------------------------------------------------------------------
// per row block: the partial fc weight and bias gradients (= gD[fc.w .. fc.b]);
// conv4's and conv5's weight gradients are block jobs of the next launch, over
// the z4 / z5 / a4 rows this kernel stores (DtOut)
constexpr int DT_SLAB = 64 + 1;
constexpr int DT_SLAB_LD = (DT_SLAB + 3) & ~3;  // slab stride: 16-byte aligned slabs

struct DiscTailLds {
  float w4[64 * 260];          // conv4 weight [64][256], padded rows
  float w5[64 * 68];           // conv5 weight [64][64]
  float wf[64];                // fc weight [1][64]
  float b4[64], b5[64], bf[4];
  alignas(16) float x3[TR * 260];   // conv3 output rows (conv4 input)
  alignas(16) float a4[TR * 68];
  float a5[TR * 68];
  float out[TR * 4];
  alignas(16) float z5[TR * 68];
  alignas(16) float z4[TR * 68];
  alignas(16) float scratch[16 * 256];
};

__global__ void __launch_bounds__(TT)
k_disc_tail(const float* __restrict__ d3, int B, const float* __restrict__ w4,
            const float* __restrict__ b4, const float* __restrict__ w5,
            const float* __restrict__ b5, const float* __restrict__ wf,
            const float* __restrict__ bf, const float* __restrict__ soft_gt,
            const float* __restrict__ soft_nogt, const int32_t* __restrict__ step, uint64_t seed,
            float lambda_adv, float* __restrict__ dd3, float* __restrict__ slabs,
            float* __restrict__ lpart3, float* __restrict__ dout, const int32_t* __restrict__ gidx,
            int C, int N, int* __restrict__ sortrec, float* __restrict__ z4g,
            float* __restrict__ z5g, float* __restrict__ a4g, int lab_off) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  DiscTailLds& L = *reinterpret_cast<DiscTailLds*>(smem);
  const int tid = threadIdx.x;
  const int R = 3 * B, nrb = (R + TR - 1) / TR;
  if ((int)blockIdx.x >= nrb) {
    // the feature backward's hit sort (feat_sort.h) on the CUs this launch
    // leaves idle: two (cloud, chunk) records per workgroup, one per half
    static_assert(TT == 2 * FS_T && sizeof(DiscTailLds) >= 2 * sizeof(SortLds), "sort geometry");
    const int nch = (N + FS_PCH - 1) / FS_PCH, half = tid / FS_T;
    const int id = 2 * ((int)blockIdx.x - nrb) + half, cc = id / nch, ch = id % nch;
    SortLds& S = reinterpret_cast<SortLds*>(smem)[half];
    const bool valid = cc < C;
    chunk_sort(gidx + (size_t)(valid ? cc : 0) * FS_MAXO, FS_MAXO, ch * FS_PCH, tid % FS_T, valid,
               S, sortrec + (size_t)id * FS_REC);
    return;
  }
  TSTAMP(1, 0);
  // every argument the row blocks read, in one round of scalar loads (a late
  // first use costs a dependent kernarg round trip, common.h)
  kernarg_prefetch(d3, w4, b4, w5, b5, wf, bf, soft_gt, soft_nogt, step, seed, lambda_adv, dd3,
                   slabs, lpart3, dout, z4g, z5g, a4g, lab_off);
  const int r0 = blockIdx.x * TR, nrows = min(TR, R - r0);
  // per-row label inputs, fetched with the weights (thread t < 16: row r0 + t)
  float ysoft = 0.f;
  uint32_t stepv = 0;
  if (tid < TR) {
    const int m = r0 + tid;
    if (m < B && soft_gt) ysoft = soft_gt[m];
    else if (m >= B && m < 2 * B && soft_nogt) ysoft = soft_nogt[m - B];
    if (m < 2 * B && ((m < B && !soft_gt) || (m >= B && !soft_nogt))) stepv = (uint32_t)*step;
  }
  if (tid == 0) L.bf[0] = bf[0];
  {
    const Fill f[6] = {{L.w4, 260, w4, 64, 256, 64}, {L.w5, 68, w5, 64, 64, 64},
                       {L.wf, 64, wf, 1, 64, 1}, {L.x3, 260, d3 + (size_t)r0 * 256, TR, 256, nrows},
                       {L.b4, 64, b4, 1, 64, 1}, {L.b5, 64, b5, 1, 64, 1}};
    lds_fill(f);  // 6192 float4: <= 7 per thread
  }
  __syncthreads();
  TSTAMP(1, 1);
  rows_layer<256, 64, B_OK, ACT_LRELU, 64>(L.x3, 260, L.w4, 260, L.b4, L.a4, 68, L.scratch);
  TSTAMP(1, 2);
  rows_layer<64, 64, B_OK, ACT_LRELU, 16>(L.a4, 68, L.w5, 68, L.b5, L.a5, 68, L.scratch);
  TSTAMP(1, 3);
  rows_layer<64, 1, B_OK, ACT_NONE, 4>(L.a5, 68, L.wf, 64, L.bf, L.out, 4, L.scratch);
  TSTAMP(1, 4);
  // BCEWithLogits terms (train_classification.py:200): rows [0,B) D(lsm_gt) vs U(0.7,1.05),
  // [B,2B) D(lsm_nogt) vs U(0,0.305), [2B,3B) adversarial vs 1
  float l0 = 0.f, l1 = 0.f, l2 = 0.f;
  if (tid < TR) {
    const int m = r0 + tid;
    float g = 0.f;
    if (m < R) {
      const float x = L.out[tid * 4];
      if (dout) dout[m] = x;  // the D logits (run_training_semi's confidence, trainer.py:717)
      float y, f;
      if (m < B) {
        y = soft_gt ? ysoft : 0.7f + 0.35f * rng_uniform(seed, stepv, RNG_LABEL_GT, (uint32_t)(m + lab_off));
        f = 0.5f;
      } else if (m < 2 * B) {
        y = soft_nogt ? ysoft
                      : 0.305f * rng_uniform(seed, stepv, RNG_LABEL_NOGT,
                                                  (uint32_t)(m - B + lab_off));
        f = 0.5f;
      } else {
        y = 1.f;
        f = lambda_adv;
      }
      g = f * (1.f / (1.f + expf(-x)) - y) / (float)B;
      const float bce = fmaxf(x, 0.f) - x * y + log1pf(expf(-fabsf(x)));
      if (m < B) l1 = bce;
      else if (m < 2 * B) l2 = bce;
      else l0 = bce;
    }
    L.out[tid * 4 + 1] = g;
  }
  if (tid < 64) {  // the block's three loss sums: a fixed butterfly over wave 0 (lanes >= TR add 0)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      l0 += __shfl_xor(l0, o);
      l1 += __shfl_xor(l1, o);
      l2 += __shfl_xor(l2, o);
    }
    if (tid == 0) {
      lpart3[blockIdx.x * 3 + 0] = l0;
      lpart3[blockIdx.x * 3 + 1] = l1;
      lpart3[blockIdx.x * 3 + 2] = l2;
    }
  }
  __syncthreads();
  // backward: fc (dz = dL/dout, no activation), conv5, conv4
  TSTAMP(1, 5);
  rows_layer<1, 64, B_KO, ACT_NONE>(L.out + 1, 4, L.wf, 64, nullptr, L.z5, 68, L.scratch);
  TSTAMP(1, 6);
  for (int e = tid; e < TR * 64; e += TT) {
    const int row = e >> 6, col = e & 63;
    L.z5[row * 68 + col] *= act_bwd(L.a5[row * 68 + col], ACT_LRELU);
  }
  __syncthreads();
  rows_layer<64, 64, B_KO, ACT_NONE, 16>(L.z5, 68, L.w5, 68, nullptr, L.z4, 68, L.scratch);
  TSTAMP(1, 7);
  for (int e = tid; e < TR * 64; e += TT) {
    const int row = e >> 6, col = e & 63;
    L.z4[row * 68 + col] *= act_bwd(L.a4[row * 68 + col], ACT_LRELU);
  }
  __syncthreads();
  // stored as D conv3's dz: times lrelu'(conv3 output), which is this block's x3 rows
  rows_layer<64, 256, B_KO, ACT_NONE, 128, ACT_LRELU>(L.z4, 68, L.w4, 260, nullptr,
                                                      dd3 + (size_t)r0 * 256, 256, L.scratch,
                                                      nrows, TR, 0, OutMask{L.x3, 260, nullptr, 1.f});
  TSTAMP(1, 8);
  // weight gradients over the D-loss rows (m < 2B; the adversarial rows train
  // only the generator): conv4's and conv5's run as block jobs of the next
  // launch over the z4 / z5 / a4 rows stored here (one 16-B store per thread
  // and row array); fc's (64 + 1 values) as this block's partial slab
  if (tid < 3 * 256) {
    const int arr = tid >> 8, e = tid & 255, row = e >> 4, c4 = e & 15, m = r0 + row;
    if (m < 2 * B) {
      const float* src = arr == 0 ? L.z4 : (arr == 1 ? L.z5 : L.a4);
      float* dst = arr == 0 ? z4g : (arr == 1 ? z5g : a4g);
      *reinterpret_cast<f32x4t*>(dst + (size_t)m * 64 + 4 * c4) =
          *reinterpret_cast<const f32x4t*>(src + row * 68 + 4 * c4);
    }
  }
  float* slab = slabs + (size_t)blockIdx.x * DT_SLAB_LD;
  TSTAMP(1, 9);
  TSTAMP(1, 10);
  if (tid < 64) {
    float s = 0.f;
    for (int row = 0; row < TR; ++row)
      if (r0 + row < 2 * B) s = fmaf(L.out[row * 4 + 1], L.a5[row * 68 + tid], s);
    slab[tid] = s;
  } else if (tid == 64) {
    float s = 0.f;
    for (int row = 0; row < TR; ++row)
      if (r0 + row < 2 * B) s += L.out[row * 4 + 1];
    slab[DT_SLAB - 1] = s;
  }
}

// ---------------------------------------------------------------------------
// k_head_bwd: rows m of the 2B generator outputs (+ conv1 weight-grad blocks)
// ---------------------------------------------------------------------------
// run_training_semi's pseudo-label loss (utils/trainer.py:716-728):
//   ignore = D(lsm_nogt) <= semi_TH, semi_gt = argmax(pred_nogt) (first index),
//   l_semi = CrossEntropyLoss(ignore_index=255)(pred_nogt, semi_gt): the mean of
//   -log_softmax(pred_nogt)[semi_gt] over the kept clouds, none when all are
//   ignored; its gradient lambda_semi (softmax - onehot) / kept reaches the
//   no-GT logits next to the adversarial one.
__device__ __forceinline__ void wave_argmax40(float v, int lane, float& mx, int& am) {
  // (value, index) max over the lanes < 40, lower index on equal values
  float bv = lane < 40 ? v : -INFINITY;
  int bi = lane < 40 ? lane : 64;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  mx = bv;
  am = bi;
}

__device__ __forceinline__ int semi_kept(const float* dout, int B, float th, int lane) {
  int c = 0;
  for (int j = lane; j < B; j += 64) c += dout[2 * B + j] > th ? 1 : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  return c;
}
struct HeadBwdLds {
  float w1[512 * 48];          // discriminator conv1 weight [512][40], rows padded to 48
  alignas(16) float z1[TR * 516];
  float ddin[TR * 44];
  float dl[TR * 44];
  alignas(16) float scratch[12 * 256];
};

__global__ void __launch_bounds__(TT)
k_head_bwd(const float* __restrict__ dz1, const float* __restrict__ h2,
           const float* __restrict__ drop_mask, float drop_keep,
           const float* __restrict__ din, int B, const float* __restrict__ dw1,
           const float* __restrict__ w3, float* __restrict__ dlogits, float* __restrict__ dh2,
           float* __restrict__ gw1, float* __restrict__ gb1, const float* __restrict__ lpart,
           int nlp, const float* __restrict__ lpart3, int nlp3, float* __restrict__ losses,
           SemiArgs semi, const float* __restrict__ ddp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  HeadBwdLds& L = *reinterpret_cast<HeadBwdLds*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = 2 * B, nrb = (C + TR - 1) / TR;
  if ((int)blockIdx.x >= nrb) {
    // discriminator conv1 weight gradient over the D-loss rows [0, 2B):
    // dW[o][k] = sum_m dz[m][o] din[m][k] (dz1 stored masked by D conv2's
    // backward); wave = 16x16 tile
    const int t = ((int)blockIdx.x - nrb) * TW + wave;
    constexpr int TK = 3;  // 40 columns in 3 tiles
    if (t >= 32 * TK) return;
    const int o0 = 16 * (t / TK), k0 = 16 * (t % TK), r = lane & 15, q = lane >> 4;
    f32x4t acc = {0.f, 0.f, 0.f, 0.f};
    float s = 0.f;
    for (int m0 = 0; m0 < C; m0 += 16) {
      float a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = m0 + 4 * u + q;
        const bool vm = m < C;
        const size_t ia = (size_t)(vm ? m : 0) * 512 + o0 + r;
        const float z = dz1[ia];
        a[u] = vm ? z : 0.f;
        const bool vb = vm && k0 + r < 40;
        const float xv = din[(size_t)(vm ? m : 0) * 40 + (vb ? k0 + r : 0)];
        b[u] = vb ? xv : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc = mfma16t(a[u], b[u], acc);
        s += a[u];
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v)
      if (k0 + r < 40) gw1[(size_t)(o0 + 4 * q + v) * 40 + k0 + r] = acc[v];
    if (k0 == 0) {
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if (q == 0) gb1[o0 + r] = s;
    }
    return;
  }
  TSTAMP(2, 0);
  kernarg_prefetch(dz1, h2, drop_mask, drop_keep, din, dw1, w3, dlogits, dh2, lpart, nlp, lpart3,
                   nlp3, losses, semi.on, semi.lambda, semi.th, semi.logits, semi.dout, ddp);
  const int r0 = blockIdx.x * TR, nrows = min(TR, C - r0);
  // this wave's row of log_softmax outputs (noGT) or CE gradient (GT)
  float lsm_or_dl = 0.f;
  {
    const int m = r0 + wave;
    if (m < C && lane < 40) lsm_or_dl = m >= B ? din[(size_t)m * 40 + lane] : dlogits[(size_t)m * 40 + lane];
  }
  // this block's h2 and dropout-mask rows (the output mask of the last layer),
  // fetched now and parked in LDS once z1 is consumed: one float4 each
  f32x4 hv, mv = {1.f, 1.f, 1.f, 1.f};
  auto load_h2_mask = [&]() {
    const int row = tid >> 6, c4 = tid & 63, m = r0 + row;
    const size_t i = (size_t)(m < C ? m : 0) * 256 + 4 * c4;
    hv = *reinterpret_cast<const f32x4*>(h2 + i);
    if (drop_mask) mv = *reinterpret_cast<const f32x4*>(drop_mask + i);
  };
  if (ddp) {
    // D conv1's input gradient of the adversarial rows from the 32 column-tile
    // partials the D conv2 backward chained onto its data gradient
    // (ddp[ct][m - B][40], LinBwdExtra.chain_*): 640 threads = (row, 4
    // columns) x 4 groups of 8 tiles, summed in tile order, the groups in order
    constexpr int NCT = 512 / 16, G4 = 4, PER = NCT / G4, NIT = TR * 10;
    const bool any = r0 + TR > B;  // block-uniform: GT-only blocks need no ddin
    f32x4 pv[PER];
    const int item = tid % NIT, grp = tid / NIT, row = item / 10, j4 = item % 10, m = r0 + row;
    const bool vr = any && grp < G4 && m >= B && m < C;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const size_t i = vr ? ((size_t)(grp * PER + u) * B + (m - B)) * 40 + 4 * j4 : 0;
      pv[u] = *reinterpret_cast<const f32x4*>(ddp + i);
    }
    load_h2_mask();
    f32x4* gs = reinterpret_cast<f32x4*>(L.scratch);  // [G4][NIT]
    if (grp < G4) {
      f32x4 t = vr ? pv[0] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 1; u < PER; ++u)
        if (vr) t += pv[u];
      gs[grp * NIT + item] = t;
    }
    __syncthreads();
    TSTAMP(2, 1);
    if (tid < NIT) {
      f32x4 t = gs[item];
#pragma unroll
      for (int g = 1; g < G4; ++g) t += gs[g * NIT + item];
#pragma unroll
      for (int i = 0; i < 4; ++i) L.ddin[row * 44 + 4 * j4 + i] = t[i];
    }
    __syncthreads();
    TSTAMP(2, 2);
  } else {
    // dz of the adversarial D rows m + B (m in [B, 2B)); zero for GT rows.  The
    // row loads are issued together with the conv1 weight staging.
    f32x4 zd[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * TT, row = e >> 7, c4 = e & 127, m = r0 + row;
      const bool v = m >= B && m < C;
      const size_t i = v ? (size_t)(m + B) * 512 + 4 * c4 : 0;
      zd[u] = *reinterpret_cast<const f32x4*>(dz1 + i);
    }
    load_h2_mask();
    {
      const Fill f[1] = {{L.w1, 48, dw1, 512, 40, 512}};
      lds_fill(f);  // 5120 float4: 5 per thread
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * TT, row = e >> 7, c4 = e & 127, m = r0 + row;
      const bool v = m >= B && m < C;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        L.z1[row * 516 + 4 * c4 + i] = v ? zd[u][i] : 0.f;
    }
    __syncthreads();
    TSTAMP(2, 1);
    rows_layer<512, 40, B_KO, ACT_NONE>(L.z1, 516, L.w1, 48, nullptr, L.ddin, 44, L.scratch);
    TSTAMP(2, 2);
  }
  float* h2s = L.z1;             // [16][256], z1 is free now
  float* ms = L.z1 + TR * 256;   // [16][256]
  *reinterpret_cast<f32x4*>(h2s + 4 * tid) = hv;
  *reinterpret_cast<f32x4*>(ms + 4 * tid) = mv;
  // log_softmax backward (noGT rows) / the CE gradient of the GT rows
  {
    const int row = wave, m = r0 + row;
    float dl = 0.f;
    if (m >= B && m < C) {
      const float g = lane < 40 ? L.ddin[row * 44 + lane] : 0.f;
      float s = g;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
      if (lane < 40) dl = g - expf(lsm_or_dl) * s;
      if (semi.on) {
        const int kept = semi_kept(semi.dout, B, semi.th, lane);
        if (kept > 0 && semi.dout[m + B] > semi.th) {
          float mx;
          int am;
          wave_argmax40(lane < 40 ? semi.logits[(size_t)m * 40 + lane] : 0.f, lane, mx, am);
          if (lane < 40)
            dl += semi.lambda / (float)kept * (expf(lsm_or_dl) - (lane == am ? 1.f : 0.f));
        }
      }
      if (lane < 40) dlogits[(size_t)m * 40 + lane] = dl;
    } else if (m < B && lane < 40) {
      dl = lsm_or_dl;
    }
    if (lane < 40) L.dl[row * 44 + lane] = dl;
  }
  __syncthreads();
  TSTAMP(2, 3);
  // stored as fc2's dz: times relu'(h2) and the dropout mask x 1/(1-p)
  rows_layer<40, 256, B_KO, ACT_NONE, 128, ACT_RELU>(
      L.dl, 44, w3, 256, nullptr, dh2 + (size_t)r0 * 256, 256, nullptr, nrows, TR, 0,
      OutMask{h2s, 256, drop_mask ? ms : nullptr, drop_keep});
  TSTAMP(2, 4);
  if (semi.on && blockIdx.x == 0 && wave == 0) {
    // l_semi and the kept ratio (losses[4], losses[5]), rows in order
    const int kept = semi_kept(semi.dout, B, semi.th, lane);
    float sum = 0.f;
    for (int j = 0; j < B; ++j) {
      if (!(semi.dout[2 * B + j] > semi.th)) continue;
      const float x = lane < 40 ? semi.logits[(size_t)(B + j) * 40 + lane] : -INFINITY;
      float mx;
      int am;
      wave_argmax40(x, lane, mx, am);
      float e = lane < 40 ? expf(x - mx) : 0.f;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o);
      sum += logf(e);  // -log_softmax at the argmax = log sum exp(x - max)
    }
    if (lane == 0) {
      losses[4] = kept > 0 ? sum / (float)kept : 0.f;
      losses[5] = (float)kept / (float)B;
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    // losses: CE mean, adversarial BCE mean, 0.5 x D-loss means (row-block order)
    float s = 0.f;
    for (int i = 0; i < nlp; ++i) s += lpart[i];
    losses[0] = s / (float)B;
    float a = 0.f, g = 0.f, n = 0.f;
    for (int i = 0; i < nlp3; ++i) {
      a += lpart3[3 * i];
      g += lpart3[3 * i + 1];
      n += lpart3[3 * i + 2];
    }
    losses[1] = a / (float)B;
    losses[2] = 0.5f * g / (float)B;
    losses[3] = 0.5f * n / (float)B;
  }
}

// ---------------------------------------------------------------------------
// k_cls_head: run_training_pointnet_cls's head end (utils/trainer.py:254-268):
// fc3 (models/pointnet.py:202), log_softmax + CrossEntropyLoss
// (train_classification.py:199), lambda_cls x its gradient and fc3's input
// gradient - stored as fc2's dz (relu'(h2) x dropout mask x keep) - one
// workgroup per 16 rows, in place of three launches.  fc3's weight gradient
// and the batch mean of the CE (rowloss[r] = CE_r / B, summed in row order)
// ride in fc2's backward launch (a LinBwdJob over dlogits x h2, its slab sum).
// ---------------------------------------------------------------------------
struct ClsHeadLds {
  float w3[40 * 260];                 // fc3 weight [40][256], padded rows
  float b3[40];
  alignas(16) float h2[TR * 260];     // the block's fc2 output rows
  alignas(16) float g[TR * 260];      // relu'(h2) x dropout mask x keep
  float lg[TR * 44];                  // logits
  float dl[TR * 44];                  // lambda dCE / dlogits
  float rl[TR];
  int lab[TR];
  alignas(16) float scratch[12 * 256];
};

__global__ void __launch_bounds__(TT)
k_cls_head(const float* __restrict__ h2, const float* __restrict__ drop_mask, float keep,
           const float* __restrict__ w3, const float* __restrict__ b3,
           const int64_t* __restrict__ labels, int B, float lambda_cls, float* __restrict__ logits,
           float* __restrict__ dlogits, float* __restrict__ dz2, float* __restrict__ rowloss,
           const int32_t* __restrict__ gidx, int C, int N, int* __restrict__ sortrec) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nrb = (B + TR - 1) / TR;
  if ((int)blockIdx.x >= nrb) {
    // the feature backward's hit sort (feat_sort.h) on the CUs this launch
    // leaves idle, as k_disc_tail does for the adversarial step
    static_assert(TT == 2 * FS_T && sizeof(ClsHeadLds) >= 2 * sizeof(SortLds), "sort geometry");
    const int nch = (N + FS_PCH - 1) / FS_PCH, half = tid / FS_T;
    const int id = 2 * ((int)blockIdx.x - nrb) + half, cc = id / nch, ch = id % nch;
    SortLds& S = reinterpret_cast<SortLds*>(smem)[half];
    const bool valid = cc < C;
    chunk_sort(gidx + (size_t)(valid ? cc : 0) * FS_MAXO, FS_MAXO, ch * FS_PCH, tid % FS_T, valid,
               S, sortrec + (size_t)id * FS_REC);
    return;
  }
  ClsHeadLds& L = *reinterpret_cast<ClsHeadLds*>(smem);
  kernarg_prefetch(h2, drop_mask, keep, w3, b3, labels, lambda_cls, logits, dlogits, dz2, rowloss);
  const int r0 = blockIdx.x * TR, nr = min(TR, B - r0);
  TSTAMP(0, 0);
  {
    const Fill f[4] = {{L.h2, 260, h2 + (size_t)r0 * 256, TR, 256, nr},
                       {L.g, 260, drop_mask + (size_t)r0 * 256, TR, 256, drop_mask ? nr : 0},
                       {L.w3, 260, w3, 40, 256, 40}, {L.b3, 40, b3, 1, 40, 1}};
    if (tid < nr) L.lab[tid] = (int)labels[r0 + tid];
    lds_fill<4, 5, false>(f);  // 4618 float4: <= 5 per thread
  }
  __syncthreads();
  TSTAMP(0, 1);
  // g = relu'(h2) x mask x keep (the mask rows were staged into g)
  for (int e = tid; e < TR * 256; e += TT) {
    const int r = e >> 8, k = e & 255;
    const float m = drop_mask ? L.g[r * 260 + k] * keep : 1.f;
    L.g[r * 260 + k] = L.h2[r * 260 + k] > 0.f ? m : 0.f;
  }
  // fc3: reduction chunks of 64 (as k_head_fwd)
  rows_layer<256, 40, B_OK, ACT_NONE, 64>(L.h2, 260, L.w3, 260, L.b3, L.lg, 44, L.scratch);
  TSTAMP(0, 2);
  // log_softmax, CE and its gradient (as k_row_ce_wave): one wave per row
  {
    const int row = wave;
    const float v = lane < 40 ? L.lg[row * 44 + lane] : -INFINITY;
    float mx = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    const float e = lane < 40 ? expf(v - mx) : 0.f;
    float se = e;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const float lse = mx + logf(se);
    float dl = 0.f;
    if (row < nr) {
      const int y = L.lab[row];
      dl = (expf(v - lse) - (lane == y ? 1.f : 0.f)) * (lambda_cls / (float)B);
      const float rloss = lse - __shfl(v, y);
      if (lane < 40) {
        logits[(size_t)(r0 + row) * 40 + lane] = v;
        dlogits[(size_t)(r0 + row) * 40 + lane] = dl;
      }
      if (lane == 0) rowloss[r0 + row] = rloss / (float)B;
    }
    if (lane < 40) L.dl[row * 44 + lane] = dl;
  }
  __syncthreads();
  TSTAMP(0, 3);
  // fc3 input gradient, stored as fc2's dz: dl W3 x g
  rows_layer<40, 256, B_KO, ACT_NONE>(L.dl, 44, L.w3, 260, nullptr, dz2 + (size_t)r0 * 256, 256,
                                      nullptr, nr, TR, 0, OutMask{L.g, 260, L.g, 1.f});
  TSTAMP(0, 4);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <typename K>
static int set_lds(K kern, size_t bytes, const char* what) {
  static_assert(sizeof(K) > 0, "");
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
    set_error("%s: cannot reserve %zu bytes of LDS", what, bytes);
    return PCADV_EHIP;
  }
  return PCADV_OK;
}

size_t disc_tail_slab_floats() { return DT_SLAB_LD; }  // per row block (stride)
int disc_tail_slab_n() { return DT_SLAB; }             // floats reduced into gD
int head_rowblocks(int B) { return (2 * B + TR - 1) / TR; }
int disc_rowblocks(int B) { return (3 * B + TR - 1) / TR; }

int launch_head_fwd(const float* h2, const float* w3, const float* b3, const int64_t* labels, int B,
                    float lambda_cls, float* logits, float* dlogits, float* din, const float* dw1,
                    const float* db1, float* d1, float* lpart, hipStream_t s) {
  static bool once = false;
  if (!once) {
    if (set_lds(k_head_fwd, sizeof(HeadFwdLds), "head_fwd") != PCADV_OK) return PCADV_EHIP;
    once = true;
  }
  hipLaunchKernelGGL(k_head_fwd, dim3(head_rowblocks(B) * HF_SPLIT), dim3(TT), sizeof(HeadFwdLds), s, h2, w3,
                     b3, labels, B, lambda_cls, logits, dlogits, din, dw1, db1, d1, lpart);
  PC_HIP_CHECK_LAUNCH("k_head_fwd");
  return PCADV_OK;
}

// sortrec (optional): also run the feature backward's hit sort over the C
// clouds' argmax gidx [C][1024] into sortrec (feat_sort_record_ints(C, N))
int launch_cls_head(const float* h2, const float* drop_mask, float drop_p, const float* w3,
                    const float* b3, const int64_t* labels, int B, float lambda_cls, float* logits,
                    float* dlogits, float* dz2, float* rowloss, hipStream_t s,
                    const int32_t* gidx, int C, int N, int* sortrec) {
  static bool once = false;
  if (!once) {
    if (set_lds(k_cls_head, sizeof(ClsHeadLds), "cls_head") != PCADV_OK) return PCADV_EHIP;
    once = true;
  }
  PC_REQUIRE(B > 0 && h2 && w3 && b3 && labels && logits && dlogits && dz2 && rowloss,
             "cls_head: bad arguments");
  PC_REQUIRE(!sortrec || (gidx && C > 0 && N > 0), "cls_head: the hit sort needs gidx, C and N");
  const int nsort = sortrec ? (C * ((N + FS_PCH - 1) / FS_PCH) + 1) / 2 : 0;
  const float keep = 1.0f / (1.0f - drop_p);  // as the linear kernels' dropout scale
  hipLaunchKernelGGL(k_cls_head, dim3((B + TR - 1) / TR + nsort), dim3(TT), sizeof(ClsHeadLds), s,
                     h2, drop_mask, keep, w3, b3, labels, B, lambda_cls, logits, dlogits, dz2,
                     rowloss, gidx, C, N, sortrec);
  PC_HIP_CHECK_LAUNCH("k_cls_head");
  return PCADV_OK;
}

size_t feat_sort_record_ints(int C, int N) { return (size_t)C * ((N + FS_PCH - 1) / FS_PCH) * FS_REC; }

// sortrec (optional): also run the feature backward's hit sort over the C
// clouds' argmax gidx [C][1024] into sortrec (feat_sort_record_ints(C, N))
int launch_disc_tail(const float* d3, int B, const float* w4, const float* b4, const float* w5,
                     const float* b5, const float* wf, const float* bf, const float* soft_gt,
                     const float* soft_nogt, const int32_t* step, uint64_t seed, float lambda_adv,
                     float* dd3, float* slabs, float* lpart3, float* dout, hipStream_t s,
                     const int32_t* gidx, int C, int N, int* sortrec, float* z4g, float* z5g,
                     float* a4g, int lab_off) {
  static bool once = false;
  if (!once) {
    if (set_lds(k_disc_tail, sizeof(DiscTailLds), "disc_tail") != PCADV_OK) return PCADV_EHIP;
    once = true;
  }
  PC_REQUIRE(!sortrec || (gidx && C > 0 && N > 0), "disc_tail: the hit sort needs gidx, C and N");
  const int nsort = sortrec ? (C * ((N + FS_PCH - 1) / FS_PCH) + 1) / 2 : 0;
  hipLaunchKernelGGL(k_disc_tail, dim3(disc_rowblocks(B) + nsort), dim3(TT), sizeof(DiscTailLds), s,
                     d3, B, w4, b4, w5, b5, wf, bf, soft_gt, soft_nogt, step, seed, lambda_adv, dd3,
                     slabs, lpart3, dout, gidx, C, N, sortrec, z4g, z5g, a4g, lab_off);
  PC_HIP_CHECK_LAUNCH("k_disc_tail");
  return PCADV_OK;
}

int launch_head_bwd(const float* dz1, const float* h2, const float* drop_mask, float drop_p,
                    const float* din, int B, const float* dw1,
                    const float* w3, float* dlogits, float* dh2, float* gw1, float* gb1,
                    const float* lpart, const float* lpart3, float* losses, int semi,
                    float lambda_semi, float semi_th, const float* logits, const float* dout,
                    hipStream_t s, const float* ddp) {
  static bool once = false;
  if (!once) {
    if (set_lds(k_head_bwd, sizeof(HeadBwdLds), "head_bwd") != PCADV_OK) return PCADV_EHIP;
    once = true;
  }
  // gw1 = nullptr: D conv1's weight gradient is computed elsewhere (the
  // adversarial step runs it as a block job of the fc2 backward launch)
  const int nrb = head_rowblocks(B), nwb = gw1 ? (32 * 3 + TW - 1) / TW : 0;
  const SemiArgs sa{semi, lambda_semi, semi_th, logits, dout};
  PC_REQUIRE(!semi || (logits && dout), "head_bwd: the semi term needs the logits and D outputs");
  const float keep = 1.0f / (1.0f - drop_p);  // as the linear kernels' dropout scale
  hipLaunchKernelGGL(k_head_bwd, dim3(nrb + nwb), dim3(TT), sizeof(HeadBwdLds), s, dz1, h2,
                     drop_mask, keep, din, B, dw1, w3, dlogits, dh2, gw1, gb1, lpart, nrb, lpart3, disc_rowblocks(B),
                     losses, sa, ddp);
  PC_HIP_CHECK_LAUNCH("k_head_bwd");
  return PCADV_OK;
}

#ifdef PCADV_STAMPS
int tail_stamps_read(uint64_t* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tail_stamps), sizeof(g_tail_stamps)) == hipSuccess
             ? PCADV_OK
             : PCADV_EHIP;
}
#endif

}  // namespace pcadv

/*
 * pcadv — MI355X-native (gfx950) PointNet adversarial-training hot path.
 *
 * C ABI of libpcadv.so.  Plain pointers and sizes only: every pointer is HIP
 * device memory owned by the caller (the library never allocates, frees or
 * retains a pointer past the call), every call is enqueued on `stream` without
 * a host sync and is safe to capture into a hipGraph.  Return value: PCADV_OK
 * or a negative error code; pcadv_last_error() then describes it
 * (thread-local).  No C++ exception crosses this boundary.
 *
 * Reference interfaces replaced (paths relative to the reference repo root,
 * YiruS/Adversarial_Learning_on_PointClouds):
 *   pcadv_feat_fwd / pcadv_feat_bwd  <- PointNetfeat.forward + autograd
 *                                       (models/pointnet.py:81-137; called from
 *                                        PointNetCls.forward :197-203)
 *   pcadv_conv_max_fwd               <- Conv1d(128->1024,1) + torch.max(dim=2)
 *                                       (models/pointnet.py:89,128-130; STN3d/STNkd
 *                                        :19,30-31 with relu before the max)
 *   pcadv_linear_fwd / _bwd          <- nn.Linear / 1x1 Conv1d on Bx Cx1 with
 *                                       ReLU / LeakyReLU(0.2) / Dropout
 *                                       (models/pointnet.py:191-202,
 *                                        models/discriminator.py:30-51)
 *   pcadv_adam                       <- torch.optim.Adam step
 *                                       (train_classification.py:110-122,
 *                                        utils/trainer.py:558-559)
 *   pcadv_gemm / _gemm_wgrad / _colsum / _conv_max_x3 / _row_ce
 *                                    <- PointNetSeg.forward + autograd + the
 *                                       per-point CrossEntropyLoss
 *                                       (models/pointnet.py:261-317,
 *                                        utils/trainer.py:310-400)
 *   pcadv_adv_step                   <- one iteration of utils/trainer.py:run_training
 *                                       (:426-559) incl. the losses of
 *                                       train_classification.py:199-200 and
 *                                       make_D_label (utils/utils.py:22-31)
 *
 * Layouts: point clouds are B x N x 3 f32 exactly as PointNetCls receives them
 * (no transpose copy); activations are point-major [cloud][point][channel];
 * weights are the reference's [out][in] (Conv1d [out,in,1] reinterpreted).
 * Parameters of the fused step live in one flat f32 buffer per network in
 * state_dict order (offsets below).
 */
#ifndef PCADV_H
#define PCADV_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCADV_OK 0
#define PCADV_EINVAL (-1)
#define PCADV_EHIP (-2)

#define PCADV_ACT_NONE 0
#define PCADV_ACT_RELU 1
#define PCADV_ACT_LRELU 2 /* LeakyReLU(negative_slope=0.2), discriminator.py:39 */

/* channel widths of the cls generator (models/pointnet.py:86-89,191-193) */
#define PCADV_C1 64
#define PCADV_C2 64
#define PCADV_C3 128
#define PCADV_C4 1024

/* flat parameter layout of PointNetCls(k=40) in state_dict order */
enum {
  PCADV_G_CONV1_W = 0, PCADV_G_CONV1_B = 192,
  PCADV_G_CONV2_W = 256, PCADV_G_CONV2_B = 4352,
  PCADV_G_CONV3_W = 4416, PCADV_G_CONV3_B = 12608,
  PCADV_G_CONV4_W = 12736, PCADV_G_CONV4_B = 143808,
  PCADV_G_FC1_W = 144832, PCADV_G_FC1_B = 669120,
  PCADV_G_FC2_W = 669632, PCADV_G_FC2_B = 800704,
  PCADV_G_FC3_W = 800960, PCADV_G_FC3_B = 811200,
  PCADV_G_NUMEL = 811240
};
/* flat parameter layout of DeepConvDiscNet(40, 1) in state_dict order */
enum {
  PCADV_D_CONV1_W = 0, PCADV_D_CONV1_B = 20480,
  PCADV_D_CONV2_W = 20992, PCADV_D_CONV2_B = 152064,
  PCADV_D_CONV3_W = 152320, PCADV_D_CONV3_B = 217856,
  PCADV_D_CONV4_W = 218112, PCADV_D_CONV4_B = 234496,
  PCADV_D_CONV5_W = 234560, PCADV_D_CONV5_B = 238656,
  PCADV_D_FC_W = 238720, PCADV_D_FC_B = 238784,
  PCADV_D_NUMEL = 238785
};

const char* pcadv_last_error(void);
int pcadv_abi_version(void);

/* ---- PointNetfeat (feature_transform=False) -------------------------------
 * pts [C][N][3]; w1 [64][3], w2 [64][64], w3 [128][64], w4 [1024][128] + biases.
 * One fused pass (conv1..conv4 + max): writes x3 [C][N][128] (post-ReLU conv3
 * output, read by the backward), gmax [C][1024] (x_global, pointnet.py:129-130,
 * an exact f32 dot product) and gidx [C][1024] (argmax over points, first index
 * on ties as torch.max on CPU).  conv1/conv2 are computed in f32, conv3 as six
 * bf16 split products (f32-level); conv4 screens the points with three bf16
 * MFMAs per product (|err| <= ~3 2^-16 sum|x w|) and re-evaluates the top two
 * points of every channel in exact f32, ranked by those values. */
size_t pcadv_feat_fwd_workspace_bytes(int C, int N);
int pcadv_feat_fwd(const float* pts, int C, int N,
                   const float* w1, const float* b1, const float* w2, const float* b2,
                   const float* w3, const float* b3, const float* w4, const float* b4,
                   float* x3, float* gmax, int32_t* gidx,
                   void* workspace, size_t workspace_bytes, hipStream_t stream);

/* pcadv_feat_fwd in bf16 mode (BASELINE configs[1]'s "bf16"): conv3 and conv4
 * multiply bf16-rounded operands with f32 accumulation (one MFMA product each);
 * gmax is the winner's bf16-product value (low 6 bits of its screening key
 * dropped), gidx its point (first index on equal keys).  conv1/conv2 stay f32
 * (the backward's recompute of x1/x2 is bitwise).  x3 is stored as bf16
 * [C][N][128] (2 bytes per element, the rounding conv4 applies to it; ABI
 * version 10): pcadv_feat_bwd takes it widened to f32. */
int pcadv_feat_fwd_bf16(const float* pts, int C, int N,
                        const float* w1, const float* b1, const float* w2, const float* b2,
                        const float* w3, const float* b3, const float* w4, const float* b4,
                        void* x3, float* gmax, int32_t* gidx,
                        void* workspace, size_t workspace_bytes, hipStream_t stream);

/* The second launch of pcadv_feat_fwd alone: conv4 (128 -> 1024, no ReLU) +
 * torch.max over the points (models/pointnet.py:128-130) of given conv3
 * activations x3 [C][N][128] -> gmax, gidx [C][1024]; precision 0 = f32-level
 * (as pcadv_feat_fwd), 1 = bf16 over an f32 x3, 2 = bf16 over a bf16 x3 (as
 * pcadv_feat_fwd_bf16 runs it on the x3 it stores; ABI version 10). */
int pcadv_conv4_max(const void* x3, int C, int N, const float* w4, const float* b4,
                    float* gmax, int32_t* gidx, int precision, hipStream_t stream);

/* Bytes of workspace pcadv_feat_bwd needs for C clouds of N points. */
size_t pcadv_feat_bwd_workspace_bytes(int C, int N);

/* Autograd of pcadv_feat_fwd: dgmax [C][1024] -> dw1..db4 (overwritten).
 * The max-pool backward is sparse (each channel's gradient goes to its argmax
 * point), equal to torch's MaxBackward for unique maxima; conv1/conv2 outputs
 * of the points that receive gradient are recomputed from pts. */
int pcadv_feat_bwd(const float* dgmax, const int32_t* gidx, const float* pts, int C, int N,
                   const float* w1, const float* b1, const float* w2, const float* b2,
                   const float* w3, const float* w4, const float* x3,
                   float* dw1, float* db1, float* dw2, float* db2,
                   float* dw3, float* db3, float* dw4, float* db4,
                   void* workspace, size_t workspace_bytes, hipStream_t stream);

/* Generic 1x1-conv (K=128 -> O, O % 128 == 0) + max over points.
 * relu_before_max=1 for the T-Nets (pointnet.py:30-31,63-64).  O = 1024 runs
 * on the fused forward's k_conv4_max (split-product screen, every winner
 * re-evaluated in exact f32; with the ReLU, an all-negative channel's argmax
 * is point 0, as torch.max over the zeros gives); other O on an f32 kernel. */
int pcadv_conv_max_fwd(const float* x, int C, int N, int K, const float* w, const float* b,
                       int O, int relu_before_max, float* gmax, int32_t* gidx,
                       hipStream_t stream);

/* ---- point-wise layers: the feature-transform path --------------------------
 * (PointNetCls(feature_transform=True): PointNetfeat conv1/conv2/conv3 with the
 * STNkd(64) transform, models/pointnet.py:46-79,109-122.)  Rows are points,
 * point-major [M][C].
 *
 * pcadv_pw_fwd: y[M][O] = act(x[M][K] W^T + b) (b may be NULL), K in {3, 64,
 * 128}, O % 32 == 0, act NONE/RELU.  W is the Conv1d weight [O][K], or with
 * w_kmajor=1 a [K][O] matrix (y = x T: the feature-transform bmm,
 * pointnet.py:120-121); rows_per_w > 0 (a multiple of 64) uses one matrix per
 * rows_per_w rows (one per cloud, W + cloud * O * K). */
int pcadv_pw_fwd(const float* x, int M, int K, const float* w, const float* b, int O, int act,
                 int w_kmajor, int rows_per_w, float* y, hipStream_t stream);

/* pcadv_pw_chain: n consecutive pcadv_pw_fwd layers in ONE launch (layer i's
 * input is layer i-1's output, layer 0's is x[M][K]); every layer's y is
 * written, bitwise what the per-layer pcadv_pw_fwd calls write.  Instantiated
 * for the feature-transform extractor (models/pointnet.py:115-122, :57-60):
 * K = 3 -> 64, 64, 64, 128 (conv1, conv2, STNkd conv1, STNkd conv2) and
 * K = 64 -> 64, 128 (x2 T, conv3); other shapes return PCADV_EINVAL. ABI 9. */
#define PCADV_PW_CHAIN_MAX 4
typedef struct pcadv_pw_layer {
  const float* w; /* [O][K] Conv1d weight, or [K][O] with w_kmajor = 1 */
  const float* b; /* bias [O] or NULL */
  float* y;       /* output [M][O] */
  int O;
  int act;        /* PCADV_ACT_NONE / PCADV_ACT_RELU */
  int w_kmajor;
  int rows_per_w; /* 0, or a multiple of 64: one matrix per rows_per_w rows */
} pcadv_pw_layer;
int pcadv_pw_chain(const float* x, int M, int K, const pcadv_pw_layer* layers, int n,
                   hipStream_t stream);

/* dx[M][K] (+)= (dy * act'(y)) W  (y = that layer's output; O in {64, 128},
 * K % 32 == 0); accumulate=1 adds into dx. */
int pcadv_pw_bwd_data(const float* dy, const float* y, int act, int M, int O, const float* w,
                      int K, int w_kmajor, int rows_per_w, float* dx, int accumulate,
                      hipStream_t stream);

/* dW = sum over rows of (dy * act'(y))^T x and db (NULL: skipped), per group
 * of rows_per_group rows (0: all rows; a multiple of 256 dividing M): dw holds
 * M / rows_per_group matrices, [O][K] or with dw_kmajor=1 [K][O] (dT of the
 * bmm).  O in {64, 128}, K in {3, 64, 128}.  Deterministic (fixed-order
 * reduction over 256-row slabs in the workspace). */
size_t pcadv_pw_bwd_weight_workspace_bytes(int M, int O, int K);
int pcadv_pw_bwd_weight(const float* dy, const float* y, int act, const float* x, int M, int O,
                        int K, int rows_per_group, int dw_kmajor, float* dw, float* db,
                        void* workspace, size_t workspace_bytes, hipStream_t stream);

/* The deferred form of pcadv_pw_bwd_weight (rows_per_group = 0, dw [O][K]):
 * pcadv_pw_bwd_weight with dw = db = NULL writes only the per-slab partial sums
 * into its workspace; pcadv_pw_wgrad_finish then sums the slabs of up to 8
 * such weight gradients (each job: that call's workspace, M, O, K, and the
 * dw / db to write) in ONE launch, bitwise the per-call sums.  The
 * feature-transform step's backward finishes its five parameter gradients
 * this way.  ABI version 8. */
typedef struct pcadv_pw_wgrad_job {
  const void* slabs;
  int M, O, K;
  float* dw;
  float* db;
} pcadv_pw_wgrad_job;
int pcadv_pw_wgrad_finish(const pcadv_pw_wgrad_job* jobs, int njobs, hipStream_t stream);

/* Backward of pcadv_conv_max_fwd: each channel's gradient goes to its argmax
 * point (times [gmax > 0] when gmax_relu is given: the ReLU before the max of
 * the T-Nets, pointnet.py:30-31,63-64).  dw [O][K], db [O] (may be NULL), dx
 * [C][N][K] (NULL: skipped; rows of points without hits are written as 0).
 * dx_relu (ABI 8): x is the ReLU output of the layer below and dx is stored
 * as that layer's pre-activation gradient, dx * [x > 0], so the layer's
 * backward reads no activations for its mask. */
int pcadv_conv_max_bwd(const float* dgmax, const int32_t* gidx, const float* gmax_relu,
                       const float* x, int C, int N, int K, const float* w, int O, float* dw,
                       float* db, float* dx, int dx_relu, hipStream_t stream);

/* feature_transform_regularizer (pointnet.py:345-353): norms[b] =
 * ||T_b T_b^T - I||_F and *reg = mean_b norms[b]; backward dT = *grad_reg *
 * (2 / (B norms[b])) (T T^T - I) T.  k <= 64. */
int pcadv_tnet_reg_fwd(const float* T, int B, int k, float* norms, float* reg,
                       hipStream_t stream);
int pcadv_tnet_reg_bwd(const float* T, int B, int k, const float* grad_reg, float* dT,
                       hipStream_t stream);
/* The regulariser of a training step in two launches (ABI 9): norms and
 * *reg as pcadv_tnet_reg_fwd, dT += pcadv_tnet_reg_bwd's gradient (the bmm's
 * dT accumulated in place), and *step_count += 1 when given (the fused
 * feature-transform cls step advances its count there, ahead of its Adam). */
int pcadv_tnet_reg_step(const float* T, int B, int k, float* norms, float* reg,
                        const float* grad_reg, float* dT, int32_t* step_count,
                        hipStream_t stream);

/* ---- linear / 1x1 conv on B x C x 1 ----------------------------------------
 * y[M][Nout] = act(s * (x[M][K] w[Nout][K]^T + b)), where s is the dropout
 * scale: drop_mask[M][Nout] in {0,1} times 1/(1-drop_p) when drop_mask is
 * non-NULL, else a device Philox draw keyed by (rng_seed, *rng_step) when
 * rng_step is non-NULL, else 1.  K % 4 == 0.  add_identity_k > 0 (with
 * Nout == k*k) adds the flattened k x k identity after the activation: the
 * T-Net output transform (STNkd fc3 + iden, models/pointnet.py:70-77). */
int pcadv_linear_fwd(const float* x, const float* w, const float* b, float* y,
                     int M, int Nout, int K, int act,
                     const float* drop_mask, const int32_t* rng_step, uint64_t rng_seed,
                     float drop_p, int add_identity_k, hipStream_t stream);

/* Backward of pcadv_linear_fwd.  dz = dy * act'(y) * s (y = the forward output).
 * dx[M][K] = dz w (skipped when dx is NULL); dw[Nout][K] = sum over the first
 * m_w rows of dz^T x, db[Nout] likewise (skipped when dw is NULL). */
int pcadv_linear_bwd(const float* dy, const float* y, int act,
                     const float* drop_mask, const int32_t* rng_step, uint64_t rng_seed,
                     float drop_p, const float* x, const float* w,
                     float* dx, float* dw, float* db, int M, int m_w, int Nout, int K,
                     hipStream_t stream);

/* ---- dense point-wise GEMM engine: the segmentation net ---------------------
 * (PointNetSeg, models/pointnet.py:261-317; run_training_pointnet_seg,
 * utils/trainer.py:310-400.)  Rows are points (point-major [B*N][C]); f32
 * operands are split to bf16 hi + lo and multiplied as three bf16 MFMA products
 * with f32 accumulation (relative error <= ~1.2e-5 of sum|a b|).
 *
 * pcadv_gemm: C[m][n] (+)= sum_k A[m][k] B[n][k] (+ bias[n] + bias_rows[m /
 * rows_per_group][n]), ReLU optional.  A[m][k] = a[m*lda + k] (ta = 0) or
 * a[k*lda + m] (ta = 1, only with tb = 1); B[n][k] = b[n*ldb + k] (tb = 0: a
 * weight [out][in], the forward) or b[k*ldb + n] (tb = 1: dX = dZ W).
 * accumulate = 1 adds into C.  cmask (nullable, stored like C with stride ldm)
 * then zeroes C where cmask <= 0: the producer of a data gradient applies the
 * relu' of the layer below, so every consumer reads dZ = dY relu'(Y) already
 * masked.  precise = 1 multiplies six products of hi/mid/lo splits instead
 * (f32-level accuracy; the gradients).  c_hi / c_lo (nullable, bf16, row
 * stride ldcp): the epilogue also writes C's hi / lo planes, the operand form
 * pcadv_gemm_bf2 stages without splitting. */
int pcadv_gemm(const float* a, int64_t lda, int ta, const float* b, int64_t ldb, int tb,
               float* c, int64_t ldc, int M, int N, int K, const float* bias,
               const float* bias_rows, int rows_per_group, int relu, int accumulate,
               const float* cmask, int64_t ldm, int precise, void* c_hi, void* c_lo, int64_t ldcp,
               hipStream_t stream);

/* The forward GEMM with both operands given as bf16 hi / lo planes (A [M][K],
 * B [N][K], the 2-way splits of f32 matrices made once by their producers:
 * hi = bf16(v), lo = bf16(v - hi)); bitwise the result pcadv_gemm computes
 * from the f32 matrices (precise = 0), without re-splitting every tile.
 * K % 16, lda % 8, ldb % 8, 16-B aligned planes. */
int pcadv_gemm_bf2(const void* a_hi, const void* a_lo, int64_t lda, const void* b_hi,
                   const void* b_lo, int64_t ldb, float* c, int64_t ldc, void* c_hi, void* c_lo,
                   int64_t ldcp, int M, int N, int K, const float* bias, const float* bias_rows,
                   int rows_per_group, int relu, int accumulate, const float* cmask, int64_t ldm,
                   hipStream_t stream);
/* f32 [rows][cols] (stride ld) -> its bf16 hi / lo planes (stride ldo). */
int pcadv_split_bf2(const float* x, int64_t ld, int rows, int cols, void* hi, void* lo,
                    int64_t ldo, hipStream_t stream);
/* f32 [rows][cols] (stride ld) -> its bf16 hi / mid / lo planes (stride ldo),
 * the three-way split whose six products give pcadv_gemm's precise (f32-level)
 * GEMMs; hi / mid are pcadv_split_bf2's hi / lo.  ABI 9. */
int pcadv_split_bf3(const float* x, int64_t ld, int rows, int cols, void* hi, void* mid, void* lo,
                    int64_t ldo, hipStream_t stream);
/* pcadv_gemm with precise = 1, ta = tb = 0 (C[M][N] (+)= act(A B^T + bias)),
 * B given as the hi / mid / lo planes of its three-way split ([N][K], stride
 * ldb, K % 16 == 0, 16-B aligned; pcadv_split_bf3 once per step for a weight):
 * bitwise pcadv_gemm's result without the per-tile split of B.  M > 32.
 * ABI 9 (the segmentation forward's weight operands, models/pointnet.py:
 * 282-317). */
int pcadv_gemm_b3(const float* a, int64_t lda, const void* b_hi, const void* b_mid,
                  const void* b_lo, int64_t ldb, float* c, int64_t ldc, int M, int N, int K,
                  const float* bias, const float* bias_rows, int rows_per_group, int relu,
                  int accumulate, hipStream_t stream);

/* Weight gradient dw[o][k] (row stride ldo) (+)= sum over `rows` points of
 * dz[p][o] x[p][k]: six-product (f32-level) GEMM over fixed-order slabs of the
 * point axis.  db (nullable) (+)= the column sums of dz (the bias gradient);
 * gsum (nullable, needs rows_per_group > 0 dividing rows) = the sums of dz over
 * each group of rows_per_group rows ([rows / rows_per_group][O], overwritten:
 * fc1's per-cloud sums).  Both come from the staged dz, no second pass.
 * rows_per_group (0 = one group) also sets the slab plan, so pass the same
 * value to the workspace query. */
size_t pcadv_gemm_wgrad_workspace_bytes(int rows, int O, int Kin, int rows_per_group);
int pcadv_gemm_wgrad(const float* dz, int64_t ldz, const float* x, int64_t ldx, int rows, int O,
                     int Kin, float* dw, int64_t ldo, float* db, float* gsum, int rows_per_group,
                     int accumulate, void* workspace, size_t workspace_bytes, hipStream_t stream);
/* Descriptor forms of pcadv_gemm_wgrad's and pcadv_gemm's arguments, for the
 * split / paired entry points below.  A descriptor is read during the call
 * only: the library keeps neither it nor any pointer in it. */
typedef struct pcadv_wgrad_desc {
  const float* dz; int64_t ldz; const float* x; int64_t ldx;
  int rows, O, Kin; float* dw; int64_t ldo; float* db; float* gsum;
  int rows_per_group, accumulate; void* workspace; size_t workspace_bytes;
} pcadv_wgrad_desc;
typedef struct pcadv_gemm_desc {
  const float* a; int64_t lda; int ta; const float* b; int64_t ldb; int tb;
  float* c; int64_t ldc; int M, N, K; const float* bias; const float* bias_rows;
  int rows_per_group, relu, accumulate; const float* cmask; int64_t ldm; int precise;
  void* c_hi; void* c_lo; int64_t ldcp;
} pcadv_gemm_desc;
/* pcadv_gemm_wgrad split in two calls, so that one launch can finish the slab
 * sums of many weight gradients (the seg backward's launch count, not its
 * values: bitwise pcadv_gemm_wgrad).
 * pcadv_gemm_wgrad_slabs enqueues w's slab GEMM into w->workspace (and, when
 * w->gsum is given, the per-group sums and db now); when g is non-null it also
 * enqueues the GEMM g (a data gradient: pcadv_gemm's arguments), and where both
 * have the engine's pairable forms (g: ta = 0, tb = 1, either precision, M > 32,
 * operands vectorisable: 16-B aligned rows, VEC >= 2) the two run as ONE launch, their workgroups side by side, each output bitwise its
 * own launch's.  g must neither read nor write anything w reads or writes.
 * pcadv_wgrad_finish then enqueues the remaining dw (and db) sums of n such
 * weight gradients in one launch (more launches above 16).  Between the two
 * calls the caller keeps dw, db and the workspaces alive and untouched; nothing
 * is held by the library, so a caller that abandons a backward between them
 * simply drops its descriptors. */
int pcadv_gemm_wgrad_slabs(const pcadv_wgrad_desc* w, const pcadv_gemm_desc* g,
                           hipStream_t stream);
int pcadv_wgrad_finish(const pcadv_wgrad_desc* w, int n, hipStream_t stream);
/* Weight gradient over a few rows in exact f32 (rows in order):
 * dw0[o][k] (+)= sum_{b < B} s[b][o] x0[b][k] for k < K0, and the same with
 * x1 / K1 / dw1 when x1 is given, in one launch (fc1's per-cloud columns). */
int pcadv_wgrad_small(const float* s, int64_t lds, int B, int O, const float* x0, int64_t ldx0,
                      int K0, float* dw0, const float* x1, int64_t ldx1, int K1, float* dw1,
                      int64_t ldo, int accumulate, hipStream_t stream);

/* Column sums (bias gradients): out[n] (+)= sum_m x[m][n] [ymask[m][n] > 0];
 * pcadv_group_colsum writes one row of sums per rows_per_group rows. */
size_t pcadv_colsum_workspace_bytes(int M, int N);
int pcadv_colsum(const float* x, const float* ymask, int64_t ld, int64_t ldm, int M, int N,
                 float* out, int accumulate, void* workspace, size_t workspace_bytes,
                 hipStream_t stream);
int pcadv_group_colsum(const float* x, const float* ymask, int64_t ld, int64_t ldm, int M, int N,
                       int rows_per_group, float* out, hipStream_t stream);

/* conv + (ReLU) + max over the Npts points of each of C clouds (conv6 + the
 * global max, pointnet.py:301-303): gmax [C][O], gidx [C][O] (first index on
 * ties of the f32 values; with relu the pooled value is relu(max)).  A screened
 * GEMM keeps per-128-point-tile top-2 candidates; the winner (and the
 * runner-up on near-ties) is re-evaluated as an f32 dot product of x and w. */
size_t pcadv_conv_max_x3_workspace_bytes(int C, int Npts, int O);
int pcadv_conv_max_x3(const float* x, int64_t ldx, int C, int Npts, int K, const float* w,
                      const float* b, int O, int relu, float* gmax, int32_t* gidx,
                      void* workspace, size_t workspace_bytes, hipStream_t stream);
/* The same with the screened GEMM staging x and w from their bf16 hi / lo
 * planes (x still given in f32 for the exact re-evaluation). */
int pcadv_conv_max_bf2(const float* x, int64_t ldx, const void* x_hi, const void* x_lo,
                       int64_t ldxp, int C, int Npts, int K, const float* w, const void* w_hi,
                       const void* w_lo, const float* b, int O, int relu, float* gmax,
                       int32_t* gidx, void* workspace, size_t workspace_bytes,
                       hipStream_t stream);
/* Its backward: g' = dgmax [gmax > 0]; dw [O][K] and db [O] overwritten
 * (nullable), dx rows (stride lddx, nullable, K <= 512) accumulated:
 * deterministic.  relu_x = 1 masks the dx additions by [x > 0] (x the output
 * of a ReLU layer: the gradient leaves already multiplied by its relu'). */
int pcadv_conv_max_x3_bwd(const float* dgmax, const float* gmax, const int32_t* gidx,
                          const float* x, int64_t ldx, int C, int Npts, int O, int K,
                          const float* w, float* dw, float* db, float* dx, int64_t lddx,
                          int relu_x, hipStream_t stream);

/* ---- data path: HDF5-free dataset reader -------------------
 * Replaces h5py's f['data'][:, 0:npts, :], f['label'][:], f['pid'][:, 0:npts]
 * in dataset/modelNetData.py:43-47 and dataset/shapeNetData.py:176-181 (host
 * code; no HDF5 library).  pcadv_h5_info: rank, dims[<= 8] and the stored type
 * (PCADV_H5_F32 / _F64, or PCADV_H5_INT / _UINT | byte size << 4).
 * pcadv_h5_read: the whole dataset converted to f32 or int64 (row-major), the
 * second dimension cut to its first keep1 entries when 0 < keep1 < dims[1]. */
#define PCADV_H5_F32 1
#define PCADV_H5_F64 2
#define PCADV_H5_INT 3
#define PCADV_H5_UINT 4
#define PCADV_H5_OUT_F32 0
#define PCADV_H5_OUT_I64 1
int pcadv_h5_info(const char* path, const char* name, int* rank, int64_t* dims, int* dtype);
int pcadv_h5_read(const char* path, const char* name, int out_type, int64_t keep1, void* out,
                  size_t out_bytes);

/* Batch assembly on the device: out[b] = src[idx[b]][0:npts] (+ jitter), with
 * src [n_src][src_npts][3] resident in HBM (the whole split), labels
 * src_lab [n_src][lab_width] and part ids src_seg [n_src][src_npts] (both
 * nullable) gathered alongside.  Jitter (dataset/modelNetData.py:80-91):
 * + clip(sigma * z, -clip, clip) per coordinate (sigma = 0: none), z from
 * `noise` ([B][npts][3] f64 standard normals, computed in f64 like numpy) or,
 * when noise is NULL, Philox normals keyed by (seed, *step, point), the point
 * of batch row b counted as row rng_row0 + b (0 for a one-process loader; a
 * data-parallel rank r holding rows [rB, rB + B) of each global batch passes
 * rB, so the ranks jitter exactly as one loader of the global batch would;
 * ABI version 6).  Indices must lie in [0, n_src) (checked by the caller;
 * out-of-range rows are left untouched). */
int pcadv_gather_clouds(const float* src, int64_t n_src, int npts, int src_npts,
                        const int64_t* idx, int B, const int64_t* src_lab, int lab_width,
                        const int64_t* src_seg, double sigma, double clip, const double* noise,
                        uint64_t seed, const int32_t* step, float* out, int64_t* out_lab,
                        int64_t* out_seg, int64_t rng_row0, hipStream_t stream);

/* pcadv_gather_clouds for a graph-replayed loader: batch k = *cursor of the
 * epoch order `order` (int64, k * B + b -> source cloud), so a captured graph
 * gathers a new batch on every replay with no host copy; the caller advances
 * *cursor and *step (pcadv_iter_epilogue) and rewrites `order` at each epoch
 * (DeviceCloudLoader.index_batches' order). */
int pcadv_gather_clouds_at(const float* src, int64_t n_src, int npts, int src_npts,
                           const int64_t* order, const int32_t* cursor, int B,
                           const int64_t* src_lab, int lab_width, const int64_t* src_seg,
                           double sigma, double clip, uint64_t seed, const int32_t* step,
                           float* out, int64_t* out_lab, int64_t* out_seg, int64_t rng_row0,
                           hipStream_t stream);

/* Several graph-fed loaders' pcadv_gather_clouds_at in ONE launch (the
 * training iteration's GT and no-GT batches, trainer.py): job k is exactly the
 * arguments of one pcadv_gather_clouds_at call, and its output is bitwise that
 * call's.  1 <= njobs <= 4.  ABI version 7. */
typedef struct pcadv_gather_job {
  const float* src;
  int64_t n_src;
  int npts, src_npts;
  const int64_t* order;
  const int32_t* cursor;
  int B;
  const int64_t* src_lab;
  int lab_width;
  const int64_t* src_seg;
  double sigma, clip;
  uint64_t seed;
  const int32_t* step;
  float* out;
  int64_t* out_lab;
  int64_t* out_seg;
  int64_t rng_row0;
} pcadv_gather_job;
int pcadv_gather_clouds_multi(const pcadv_gather_job* jobs, int njobs, hipStream_t stream);

/* The end of a graph-replayed training iteration (trainer.py): counters[i] += 1
 * for i < ncounters (<= 64: loaders' RNG steps and batch cursors), and, when
 * ring is given, losses[0..nl) (nl <= 32) into slot (*ring_count % slots) of the [slots][nl]
 * loss ring, then *ring_count += 1 (the host reads the ring every `slots`
 * iterations instead of copying the losses out every iteration). */
int pcadv_iter_epilogue(int32_t* counters, int ncounters, const float* losses, int nl,
                        float* ring, int slots, int32_t* ring_count, hipStream_t stream);

/* CrossEntropyLoss over rows (the per-point segmentation loss, mean over M
 * points): *loss, and dlogits = scale * dL/dlogits (same stride ld). */
size_t pcadv_row_ce_workspace_bytes(int M);
int pcadv_row_ce(const float* logits, int64_t ld, const int64_t* labels, int M, int ncls,
                 float scale, float* loss, float* dlogits, void* workspace,
                 size_t workspace_bytes, hipStream_t stream);

/* ---- Adam (torch.optim.Adam semantics, amsgrad=False, weight_decay=0) ------
 * step_count: device int32, incremented by this call (t = *step_count + 1). */
int pcadv_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
               int64_t n, int32_t* step_count, float lr, float beta1, float beta2,
               float eps, hipStream_t stream);

/* out = [a; b] (na + nb floats) and, when inc_counter is not NULL,
 * *inc_counter += 1: the feature-transform step's first launch, its GT and
 * no-GT batches as one 2B-cloud input (PointNetCls runs on each,
 * utils/trainer.py:467,490) and the iteration's step number advanced for the
 * device draws and pcadv_adam2.  ABI version 8. */
int pcadv_concat2(const float* a, int64_t na, const float* b, int64_t nb, float* out,
                  int32_t* inc_counter, hipStream_t stream);

/* Two Adam updates of one iteration in one launch (segment 1 may be empty,
 * n1 = 0), each with its own learning rate, at the step number *step_count
 * that the iteration already advanced (pcadv_adv_step part 3): t =
 * *step_count, not incremented.  The feature-transform step's optimizer.step()
 * + optimizer_D.step() (utils/trainer.py:558-559).  ABI version 8. */
int pcadv_adam2(float* p0, const float* g0, float* m0, float* v0, int64_t n0, float lr0,
                float* p1, const float* g1, float* m1, float* v1, int64_t n1, float lr1,
                const int32_t* step_count, float beta1, float beta2, float eps,
                hipStream_t stream);

/* ---- the fused adversarial step (utils/trainer.py:426-559) -------------------
 * B clouds of N points per loader.  Stochastic inputs: when drop_mask_gt /
 * drop_mask_nogt ([B][256] {0,1}) or soft_gt / soft_nogt ([B]) are NULL they are
 * drawn on device from Philox keyed by (rng_seed, *step_count), so a captured
 * graph draws fresh values each replay. */
typedef struct pcadv_adv_args {
  int B, N;
  /* inputs */
  const float* pts_gt;      /* [B][N][3] */
  const int64_t* labels;    /* [B] class ids in [0,40) */
  const float* pts_nogt;    /* [B][N][3] */
  const float* drop_mask_gt, * drop_mask_nogt;
  const float* soft_gt, * soft_nogt;
  /* generator: flat params / grads / Adam moments (PCADV_G_NUMEL floats) */
  float* g_param, * g_grad, * g_m, * g_v;
  /* discriminator (PCADV_D_NUMEL floats) */
  float* d_param, * d_grad, * d_m, * d_v;
  int32_t* step_count;      /* device: completed steps (shared by both Adams) */
  float lr_g, lr_d, beta1, beta2, eps;
  float lambda_cls, lambda_adv, drop_p;
  uint64_t rng_seed;
  int apply_adam;           /* 0: stop after the gradients (parity tests) */
  /* outputs */
  float* losses;            /* [4]: loss_cls, loss_adv, loss_D_gt, loss_D_nogt
                               ([6] with semi: + loss_semi, kept ratio) */
  float* logits;            /* [2B][40] or NULL */
  /* scratch */
  void* workspace;
  size_t workspace_bytes;
  /* run_training_semi (utils/trainer.py:611-847, :716-743): when semi != 0 the
   * generator loss gains lambda_semi * CrossEntropyLoss(ignore_index=255) of
   * the no-GT logits against their own argmax, the clouds with
   * D(log_softmax(pred_nogt)) <= semi_th ignored (no term when all are) */
  int semi;
  float lambda_semi, semi_th;
  /* 0: the whole step.  A data-parallel step may split it so the gradients
   * that are final early are all-reduced while the feature backward runs:
   * 1 = forward, losses, discriminator and head backward (every gradient
   *     except the generator's conv1..conv4, g_grad[0, PCADV_G_FC1_W));
   * 2 = the feature backward (those conv1..conv4 gradients; and both Adam
   *     updates when apply_adam) on the state part 1 left in the workspace;
   * 3 = part 1 from fc1 on, over the caller's features (feat_* below);
   *     pcadv_cls_step takes 0 or 3 (ABI 9: its head on given features). */
  int part;
  /* feature forward precision: 0 = f32-level (default), 1 = bf16 (as
   * pcadv_feat_fwd_bf16, x3 kept in bf16 for the feature backward; the head,
   * the discriminator and every backward stay f32 arithmetic).  ABI version 5;
   * the bf16 x3 since version 10. */
  int precision;
  /* Data parallelism (ABI version 6): rank rng_rank of rng_world (<= 1: one
   * process) holding GT rows [rank B, rank B + B) and no-GT rows [rank B,
   * rank B + B) of the rng_world B-cloud global batches.  The device-drawn
   * dropout masks and soft D labels are keyed by those global rows, so with
   * the same rng_seed and step count the ranks draw exactly the slices of the
   * one-process step on the global batch (the dropout row of no-GT row j is
   * rng_world B + j, as in the one-process [GT; no-GT] batch). */
  int rng_rank, rng_world;
  /* The graph-replayed training iteration's epilogue (pcadv_iter_epilogue:
   * epi_counters[0..epi_ncounters) += 1, losses[0..epi_nl) into slot
   * (*epi_ring_count % epi_slots) of the [epi_slots][epi_nl] ring, then
   * *epi_ring_count += 1) run by the step's last launch instead of a launch of
   * its own; epi_ncounters = 0 and epi_ring = NULL: none.  Not with part = 1.
   * pcadv_adv_step and pcadv_cls_step.  ABI version 7. */
  int32_t* epi_counters;
  int epi_ncounters;
  float* epi_ring;
  int epi_slots, epi_nl;
  int32_t* epi_ring_count;
  /* The step's input batches gathered by its first launch (the feature
   * forward's point loads) instead of a pcadv_gather_clouds_multi launch
   * before the step: job 0 fills pts_gt (and, with src_lab, the label rows
   * `labels` points into), job 1 pts_nogt (the adversarial step; the cls step
   * takes job 0 only).  Each job as pcadv_gather_clouds_at (device jitter, no
   * part ids) with out = the step's input buffer: bitwise that gather's
   * batch.  ngather = 0: none.  ABI version 7. */
  const pcadv_gather_job* gather;
  int ngather;
  /* A generator whose feature extractor runs outside the step (the
   * feature-transform generator, PointNetCls(feature_transform=True), built
   * from the point-wise kernels): part = 3 runs part 1's work from fc1 on
   * (fc1..fc3 + dropout, log_softmax / CE, the three discriminator passes with
   * their BCE terms, D's gradients, the head backward) on the caller's pooled
   * features feat_gmax [2B][1024] (GT clouds first) and writes dL/dgmax to
   * feat_dgmax [2B][1024].  No gather, epilogue or Adam, and *step_count is
   * NOT advanced: the caller's first launch advances it (pcadv_concat2), its
   * extractor's backward and Adam (pcadv_adam2) follow.  NULL for parts 0-2.
   * ABI version 8. */
  const float* feat_gmax;
  float* feat_dgmax;
} pcadv_adv_args;

size_t pcadv_adv_step_workspace_bytes(int B, int N);
int pcadv_adv_step(const pcadv_adv_args* args, hipStream_t stream);

/* The two Adam updates of pcadv_adv_step alone (optimizer.step() and
 * optimizer_D.step(), trainer.py:558-559), for a step that ran with
 * apply_adam = 0 and whose gradients were then all-reduced across ranks.
 * Uses the step counter already advanced by that pcadv_adv_step.  args->part
 * selects the parameters (Adam is elementwise, so parts 1 + 2 equal part 0
 * bitwise): 0 = all; 1 = those whose gradients part 1 of the step finalises
 * (g_param[PCADV_G_FC1_W, PCADV_G_NUMEL) and all of D), so they can update
 * while the conv1..conv4 bucket is still being all-reduced; 2 = the rest
 * (g_param[0, PCADV_G_FC1_W)). */
int pcadv_adv_step_adam(const pcadv_adv_args* args, hipStream_t stream);

/* One iteration of run_training_pointnet_cls (utils/trainer.py:222-268,
 * feature_transform=False; BASELINE configs[1]): PointNetCls forward on the B
 * clouds of pts_gt (labels), loss = lambda_cls * CrossEntropyLoss, backward,
 * and (apply_adam) the generator's Adam step.  Uses the generator fields of
 * pcadv_adv_args (pts_nogt, d_*, soft_*, lambda_adv, semi ignored);
 * drop_mask_gt optional (else device-drawn); losses[0] = CE; workspace as
 * pcadv_adv_step_workspace_bytes(B, N).  part = 3 (ABI 9): the head alone on
 * the caller's pooled features feat_gmax [B][1024] (fc1 .. the CE, and back to
 * feat_dgmax = dL/dgmax and the head's gradients), for the feature-transform
 * generator's step whose extractor runs outside; the caller advances
 * *step_count first (the dropout draws read it) and runs Adam. */
int pcadv_cls_step(const pcadv_adv_args* args, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PCADV_H */

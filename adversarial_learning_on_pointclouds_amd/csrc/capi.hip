// extern "C" entry points of libpcadv.so (include/pcadv.h) and the fused
// adversarial step, which enqueues the whole iteration of
// utils/trainer.py:run_training (:426-559) on one stream.
#include <cstdarg>
#include <cstdio>

#include "common.h"

#ifndef PCADV_CLS_PRESORT
#define PCADV_CLS_PRESORT 1  // A/B builds: 0 = the cls step's chunks sort their own hits
#endif

namespace pcadv {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_point_mlp3(const float*, const float*, int, int, int, const float*, const float*,
                      const float*, const float*, const float*, const float*, float*, float*,
                      float*, int32_t*, hipStream_t);
int launch_conv_max128(const float*, int, int, const float*, const float*, int, bool, float*,
                       int32_t*, hipStream_t);
size_t feat_bwd_workspace_bytes(int C, int N);
int launch_feat_bwd(const float*, const int32_t*, const float*, const float*, int, int, int,
                    const float*, const float*, const float*, const float*, const float*,
                    const float*, const float*, float*, float*, float*, float*, float*, float*,
                    float*, float*, void*, size_t, hipStream_t, uint64_t* stamps = nullptr,
                    const FinAdam* adam = nullptr, const int* sortrec = nullptr,
                    const IterEpi* epi = nullptr, int x3_bf16 = 0);
size_t feat_fwd_workspace_bytes(int C, int N);
int launch_feat_fwd_fused(const float*, const float*, int, int, int, const float*, const float*,
                          const float*, const float*, const float*, const float*, const float*,
                          const float*, float*, float*, int32_t*, int32_t*, void*, size_t,
                          hipStream_t, uint64_t* stamps = nullptr, int precision = 0,
                          const pcadv_gather_job* gather = nullptr, int ngather = 0);
int launch_conv4_max(const float*, int, int, const float*, const float*, float*, int32_t*,
                     hipStream_t, int, int relu = 0);
int launch_linear_fwd(const float*, const float*, const float*, float*, int, int, int, int,
                      const float*, const int32_t*, uint64_t, float, hipStream_t,
                      int add_identity_k = 0, float* mask_out = nullptr, int row_split = 0,
                      int row_off_lo = 0, int row_off_hi = 0);
int launch_pw_fwd(const float*, int, int, const float*, const float*, int, int, int, int, float*,
                  hipStream_t);
int launch_pw_chain(const float*, int, int, const pcadv_pw_layer*, int, hipStream_t);
int launch_pw_bwd_data(const float*, const float*, int, int, int, const float*, int, int, int,
                       float*, int, hipStream_t);
size_t pw_bwd_weight_workspace_bytes(int M, int O, int K);
int launch_pw_bwd_weight(const float*, const float*, int, const float*, int, int, int, int, int,
                         float*, float*, void*, size_t, hipStream_t);
int launch_convmax_bwd(const float*, const int32_t*, const float*, const float*, int, int, int,
                       const float*, int, float*, float*, float*, hipStream_t, int);
int launch_tnet_reg(const float*, int, int, float*, float*, const float*, float*, hipStream_t,
                    int accumulate = 0, int32_t* step_inc = nullptr);
int launch_adam2(float*, const float*, float*, float*, int64_t, float, float*, const float*,
                 float*, float*, int64_t, float, const int32_t*, int, float, float, float,
                 hipStream_t);
int launch_inc(int32_t*, hipStream_t);
int launch_pw_wgrad_finish(const pcadv_pw_wgrad_job*, int, hipStream_t);
int launch_concat2(const float*, int64_t, const float*, int64_t, float*, int32_t*, hipStream_t);
size_t disc_tail_slab_floats();
int disc_tail_slab_n();
int head_rowblocks(int B);
int disc_rowblocks(int B);
int launch_head_fwd(const float*, const float*, const float*, const int64_t*, int, float, float*,
                    float*, float*, const float*, const float*, float*, float*, hipStream_t);
int launch_disc_tail(const float*, int, const float*, const float*, const float*, const float*,
                     const float*, const float*, const float*, const float*, const int32_t*,
                     uint64_t, float, float*, float*, float*, float*, hipStream_t,
                     const int32_t* gidx, int C, int N, int* sortrec, float* z4g, float* z5g,
                     float* a4g, int lab_off = 0);
size_t feat_sort_record_ints(int C, int N);
#if defined(PCADV_C4_CERT) && PCADV_C4_CERT
int c4_cert_read(unsigned* host);
#endif
#ifdef PCADV_STAMPS
int tail_stamps_read(uint64_t* host);
int chunk_stamps_read(uint64_t* host);
int lin_stamps_read(uint64_t* host, int reset);
#endif
int launch_head_bwd(const float*, const float*, const float*, float, const float*, int,
                    const float*, const float*, float*, float*, float*, float*, const float*,
                    const float*, float*, int, float, float, const float*, const float*,
                    hipStream_t, const float*);
int launch_gemm(const float*, long long, int, const float*, long long, int, float*, long long,
                int, int, int, const float*, const float*, int, int, int, const float*, long long,
                int, void*, void*, long long, hipStream_t);
int launch_gemm_bf2(const void*, const void*, long long, const void*, const void*, long long, float*,
                    long long, void*, void*, long long, int, int, int, const float*, const float*,
                    int, int, int, const float*, long long, hipStream_t);
int launch_split_bf2(const float*, long long, int, int, void*, void*, long long, hipStream_t);
int launch_split_bf3(const float*, long long, int, int, void*, void*, void*, long long, hipStream_t);
int launch_gemm_b3(const float*, long long, const void*, const void*, const void*, long long, float*,
                   long long, int, int, int, const float*, const float*, int, int, int, hipStream_t);
size_t gemm_wgrad_workspace_bytes(int, int, int, int);
int launch_gemm_wgrad(const float*, long long, const float*, long long, int, int, int, float*,
                      long long, float*, float*, int, int, void*, size_t, hipStream_t);
int launch_gemm_wgrad_slabs(const pcadv_wgrad_desc*, const pcadv_gemm_desc*, hipStream_t);
int launch_wgrad_finish(const pcadv_wgrad_desc*, int, hipStream_t);
int launch_wgrad_small(const float*, long long, int, int, const float*, long long, int, float*,
                       const float*, long long, int, float*, long long, int, hipStream_t);
size_t colsum_workspace_bytes(int, int);
int launch_colsum(const float*, const float*, long long, long long, int, int, float*, int, void*,
                  size_t, hipStream_t);
int launch_group_colsum(const float*, const float*, long long, long long, int, int, int, float*,
                        hipStream_t);
size_t conv_max_x3_workspace_bytes(int, int, int);
int launch_conv_max_x3(const float*, long long, int, int, int, const float*, const float*, int,
                       int, float*, int32_t*, void*, size_t, hipStream_t, const void*, const void*,
                       long long, const void*, const void*);
int launch_cmx_bwd(const float*, const float*, const int32_t*, const float*, long long, int, int,
                   int, int, const float*, float*, float*, float*, long long, int, hipStream_t);
int launch_gather_clouds(const float*, int64_t, int, int, const int64_t*, int, const int64_t*, int,
                         const int64_t*, double, double, const double*, uint64_t, const int32_t*,
                         float*, int64_t*, int64_t*, hipStream_t, const int32_t* cursor = nullptr,
                         int64_t rng_row0 = 0);
int launch_iter_epilogue(int32_t*, int, const float*, int, float*, int, int32_t*, hipStream_t);
int check_iter_epi(const IterEpi&);
int launch_gather_multi(const pcadv_gather_job*, int, hipStream_t);
size_t row_ce_workspace_bytes(int);
int launch_row_ce(const float*, long long, const int64_t*, int, int, float, float*, float*, void*,
                  size_t, hipStream_t);
int launch_cls_head(const float*, const float*, float, const float*, const float*, const int64_t*,
                    int, float, float*, float*, float*, float*, hipStream_t, const int32_t*, int,
                    int, int*);

// ---- workspace carve for the fused step ------------------------------------
struct StepWs {
  float *x3, *gmax, *h1, *h2, *logits, *dlogits, *dh2, *dh1, *dgmax;
  float *din, *d1, *d2, *d3;
  float *dd3, *dd2, *dd1;
  float *z4, *z5, *a4;  // D conv4 / conv5 dz rows and conv4 output rows (k_disc_tail)
  float* ddp;           // D conv1 input-gradient partials [512 / 16][B][40] (chained)
  float *mask;
  float *lpart, *lpart3, *dslabs, *dout;
  float* rowloss;  // the cls step's per-row CE / B (k_cls_head)
  int32_t* gidx;
  int* sortrec;  // the feature backward's hit sort, done early (feat_sort.h)
  void* feat_ws;
  size_t feat_ws_bytes;
  size_t total;
};

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

static StepWs carve(int B, int N, char* base) {
  StepWs w{};
  const size_t C = 2 * (size_t)B, R = 3 * (size_t)B;
  size_t off = 0;
  auto take = [&](size_t nfloat) {
    char* p = base ? base + off : nullptr;
    off += align_up(nfloat * sizeof(float));
    return reinterpret_cast<float*>(p);
  };
  w.x3 = take(C * N * 128);  // first: Python's saved_x3() views offset 0
  w.gmax = take(C * 1024);
  w.gidx = reinterpret_cast<int32_t*>(take(C * 1024));
  w.h1 = take(C * 512);
  w.h2 = take(C * 256);
  w.logits = take(C * 40);
  w.dlogits = take(C * 40);
  w.dh2 = take(C * 256);
  w.dh1 = take(C * 512);
  w.dgmax = take(C * 1024);
  w.din = take(R * 40);
  w.d1 = take(R * 512);
  w.d2 = take(R * 256);
  w.d3 = take(R * 256);
  w.dd3 = take(R * 256);
  w.dd2 = take(R * 256);
  w.dd1 = take(R * 512);
  w.z4 = take(R * 64);
  w.z5 = take(R * 64);
  w.a4 = take(R * 64);
  w.ddp = take(32 * (size_t)B * 40);
  w.mask = take(C * 256);
  w.lpart = take(head_rowblocks(B));
  w.lpart3 = take(3 * (size_t)disc_rowblocks(B));
  w.dslabs = take((size_t)disc_rowblocks(B) * disc_tail_slab_floats());
  w.dout = take(R);
  w.rowloss = take(C);
  w.sortrec = reinterpret_cast<int*>(take(feat_sort_record_ints((int)C, N)));
  w.feat_ws_bytes = feat_bwd_workspace_bytes((int)C, N);
  if (feat_fwd_workspace_bytes((int)C, N) > w.feat_ws_bytes)
    w.feat_ws_bytes = feat_fwd_workspace_bytes((int)C, N);
  w.feat_ws = take(w.feat_ws_bytes / sizeof(float) + 1);
  w.total = off;
  return w;
}

#define PC_TRY(call)            \
  do {                          \
    int rc_ = (call);           \
    if (rc_ != PCADV_OK) return rc_; \
  } while (0)

// Adam fused into the feature backward's finishing launch (apply_adam): G's
// conv1..conv4 as their gradients are formed there, the rest of G and all of D
// in extra blocks of the same launch (their gradients are final by then).
// The fused Adam of a whole step is split by where each gradient becomes
// final: fc2, fc3 and all of D before fc1's backward launch (their update rides
// along it: early = true), fc1 before the chunk launch (its trailing
// workgroups), conv1..conv4 in the finishing launch.
#ifndef PCADV_EARLY_ADAM
#define PCADV_EARLY_ADAM 0  // A/B builds: 1 = fc2, fc3 and D ride along fc1's backward (measured slower)
#endif
// whole: the chunk launch's share when no fc1 backward ran in this call (part 2)
static FinAdam fused_adam(const pcadv_adv_args* a, bool with_d, bool early = false,
                          bool whole = false) {
  const bool split = PCADV_EARLY_ADAM && !whole;
  FinAdam f{};
  f.on = 1;
  f.gp = a->g_param; f.gm = a->g_m; f.gv = a->g_v; f.gg = a->g_grad;
  f.g_rest0 = split && early ? PCADV_G_FC2_W : PCADV_G_FC1_W;
  f.g_n = split && !early ? PCADV_G_FC2_W : PCADV_G_NUMEL;
  with_d = with_d && (!split || early);
  if (with_d) {
    f.dp = a->d_param; f.dm = a->d_m; f.dv = a->d_v; f.dg = a->d_grad;
    f.d_n = PCADV_D_NUMEL;
  }
  f.lr_g = a->lr_g; f.lr_d = a->lr_d;
  f.b1 = a->beta1; f.b2 = a->beta2; f.eps = a->eps;
  f.step_count = a->step_count;
  f.step_offset = 0;  // the step already advanced the counter (k_point_mlp)
  return f;
}

static int adv_adam(const pcadv_adv_args* a, hipStream_t s) {
  PC_REQUIRE(a && a->g_param && a->d_param && a->step_count, "adv_step_adam: bad arguments");
  PC_REQUIRE(a->part >= 0 && a->part <= 2, "adv_step_adam: part %d not in 0..2", a->part);
  if (a->part == 2)  // the generator's conv1..conv4 (the late all-reduce bucket)
    return launch_adam2(a->g_param, a->g_grad, a->g_m, a->g_v, PCADV_G_FC1_W, a->lr_g, nullptr,
                        nullptr, nullptr, nullptr, 0, 0.f, a->step_count, 0, a->beta1, a->beta2,
                        a->eps, s);
  // part 1 starts at fc1 (a multiple of 4 floats: the vector loads stay aligned)
  static_assert(PCADV_G_FC1_W % 4 == 0, "fc1 offset alignment");
  const int64_t g0 = a->part == 1 ? PCADV_G_FC1_W : 0;
  return launch_adam2(a->g_param + g0, a->g_grad + g0, a->g_m + g0, a->g_v + g0,
                      PCADV_G_NUMEL - g0, a->lr_g, a->d_param, a->d_grad, a->d_m, a->d_v,
                      PCADV_D_NUMEL, a->lr_d, a->step_count, 0, a->beta1, a->beta2, a->eps, s);
}

static int adv_head_part(const pcadv_adv_args* a, hipStream_t s, const StepWs& w, float* logits);

// pcadv_adv_args.epi_*: the iteration epilogue folded into the finishing launch
// pcadv_adv_args.gather: the labels the head reads must be the ones job 0 gathers
static int check_folded_gather(const pcadv_adv_args* a) {
  if (!a->ngather) return PCADV_OK;
  PC_REQUIRE(a->gather, "step: ngather %d without jobs", a->ngather);
  const pcadv_gather_job& j = a->gather[0];
  PC_REQUIRE(!j.src_lab || (j.lab_width == 1 && (const int64_t*)j.out_lab == a->labels),
             "step: the gathered labels (job 0, width %d) are not the step's labels", j.lab_width);
  return PCADV_OK;
}

static int step_epilogue(const pcadv_adv_args* a, IterEpi* e, bool* on) {
  *e = IterEpi{a->epi_counters, a->epi_ncounters, a->losses, a->epi_nl, a->epi_ring,
               a->epi_slots, a->epi_ring_count};
  *on = a->epi_ncounters > 0 || a->epi_ring;
  if (!*on) return PCADV_OK;
  PC_REQUIRE(a->part != 1, "adv_step: the iteration epilogue needs the finishing launch (part 0 or 2)");
  PC_REQUIRE(!a->epi_ring || a->losses, "adv_step: the loss ring needs losses");
  return check_iter_epi(*e);
}

static int adv_step(const pcadv_adv_args* a, hipStream_t s) {
  PC_REQUIRE(a && a->B > 0 && a->B <= 256 && a->N > 0, "adv_step: bad B/N");
  const int B = a->B, N = a->N, C = 2 * B;
  PC_REQUIRE(a->workspace && a->workspace_bytes >= carve(B, N, nullptr).total,
             "adv_step: workspace too small (need %zu bytes)", carve(B, N, nullptr).total);
  StepWs w = carve(B, N, static_cast<char*>(a->workspace));
  const float* G = a->g_param;
  float* gG = a->g_grad;
  float* logits = a->logits ? a->logits : w.logits;
  PC_REQUIRE(a->part >= 0 && a->part <= 3,
             "adv_step: part %d (0 whole, 1 head, 2 feature bwd, 3 head on given features)", a->part);
  PC_REQUIRE(!((a->part == 1 || a->part == 3) && a->apply_adam),
             "adv_step: part %d cannot apply Adam", a->part);
  if (a->part == 3) {
    // the caller's feature extractor (the feature-transform generator) ran
    // outside: no gather, precision or epilogue apply to this part
    PC_REQUIRE(a->feat_gmax && a->feat_dgmax, "adv_step: part 3 needs feat_gmax and feat_dgmax");
    PC_REQUIRE(!a->ngather && !a->epi_ncounters && !a->epi_ring,
               "adv_step: part 3 takes no folded gather or epilogue");
    PC_REQUIRE(a->step_count, "adv_step: step_count");
    // *step_count was advanced by the caller's first launch (pcadv_concat2),
    // as the feature forward's first launch advances it in parts 0 / 1
    return adv_head_part(a, s, w, logits);
  }
  if (a->part != 2) {
    PC_TRY(check_folded_gather(a));
    PC_TRY(adv_head_part(a, s, w, logits));
  }
  if (a->part == 1) return PCADV_OK;
  // ---- PointNetfeat backward (sparse max-pool), then optimizer.step();
  //      optimizer_D.step() (:558-559) fused into its finishing launch --------
  PC_REQUIRE(!a->apply_adam || (a->g_m && a->g_v && a->d_param && a->d_m && a->d_v),
             "adv_step: Adam buffers");
  const FinAdam fa = fused_adam(a, true, false, a->part == 2);
  IterEpi epi;
  bool epi_on;
  PC_TRY(step_epilogue(a, &epi, &epi_on));
  return launch_feat_bwd(w.dgmax, w.gidx, a->pts_gt, a->pts_nogt, B, C, N, G + PCADV_G_CONV1_W,
                         G + PCADV_G_CONV1_B, G + PCADV_G_CONV2_W, G + PCADV_G_CONV2_B,
                         G + PCADV_G_CONV3_W, G + PCADV_G_CONV4_W, w.x3,
                         gG + PCADV_G_CONV1_W, gG + PCADV_G_CONV1_B, gG + PCADV_G_CONV2_W,
                         gG + PCADV_G_CONV2_B, gG + PCADV_G_CONV3_W, gG + PCADV_G_CONV3_B,
                         gG + PCADV_G_CONV4_W, gG + PCADV_G_CONV4_B, w.feat_ws, w.feat_ws_bytes,
                         s, nullptr, a->apply_adam ? &fa : nullptr, w.sortrec,
                         epi_on ? &epi : nullptr, a->precision == 1);
}

// Part 1 of adv_step: everything before the feature backward.
static int adv_head_part(const pcadv_adv_args* a, hipStream_t s, const StepWs& w, float* logits) {
  const int B = a->B, N = a->N, C = 2 * B, R = 3 * B;
  const float* G = a->g_param;
  float* gG = a->g_grad;
  const float* D = a->d_param;
  float* gD = a->d_grad;
  const int32_t* st = a->step_count;

  // dropout: explicit masks (parity mode) are staged as one [2B][256] array
  const float* mask = nullptr;
  if (a->drop_mask_gt || a->drop_mask_nogt) {
    PC_REQUIRE(a->drop_mask_gt && a->drop_mask_nogt, "adv_step: give both dropout masks or none");
    if (hipMemcpyAsync(w.mask, a->drop_mask_gt, sizeof(float) * B * 256, hipMemcpyDeviceToDevice,
                       s) != hipSuccess ||
        hipMemcpyAsync(w.mask + (size_t)B * 256, a->drop_mask_nogt, sizeof(float) * B * 256,
                       hipMemcpyDeviceToDevice, s) != hipSuccess) {
      set_error("adv_step: mask staging copy failed");
      return PCADV_EHIP;
    }
    mask = w.mask;
  }
  const int32_t* rstep = mask ? nullptr : st;
  // device draws keyed by the global batch's rows (rank r of W holds GT rows
  // [rB, rB + B) and no-GT rows [rB, rB + B) of the W B-cloud global batches)
  const int W = a->rng_world > 1 ? a->rng_world : 1, rr = W > 1 ? a->rng_rank : 0;
  PC_REQUIRE(rr >= 0 && rr < W, "adv_step: rng_rank %d not in [0, %d)", a->rng_rank, W);

  // ---- generator forward, both loaders in one launch (:468, :490); part 3:
  //      the caller's pooled features (and no hit sort: no sparse chunks) ----
  const bool ext = a->part == 3;
  const float* gmax = ext ? a->feat_gmax : w.gmax;
  float* dgmax = ext ? a->feat_dgmax : w.dgmax;
  if (!ext)
    PC_TRY(launch_feat_fwd_fused(a->pts_gt, a->pts_nogt, B, C, N, G + PCADV_G_CONV1_W,
                                 G + PCADV_G_CONV1_B, G + PCADV_G_CONV2_W, G + PCADV_G_CONV2_B,
                                 G + PCADV_G_CONV3_W, G + PCADV_G_CONV3_B, G + PCADV_G_CONV4_W,
                                 G + PCADV_G_CONV4_B, w.x3, w.gmax, w.gidx, a->step_count,
                                 w.feat_ws, w.feat_ws_bytes, s, nullptr, a->precision, a->gather,
                                 a->ngather));
  PC_TRY(launch_linear_fwd(gmax, G + PCADV_G_FC1_W, G + PCADV_G_FC1_B, w.h1, C, 512, 1024,
                           PCADV_ACT_RELU, nullptr, nullptr, 0, 0.f, s));
  // fc2 + dropout: a device-drawn mask is stored for the backward
  PC_TRY(launch_linear_fwd(w.h1, G + PCADV_G_FC2_W, G + PCADV_G_FC2_B, w.h2, C, 256, 512,
                           PCADV_ACT_RELU, mask, rstep, a->rng_seed, a->drop_p, s, 0,
                           mask ? nullptr : w.mask, B, rr * B, (W - 1) * B + rr * B));
  const float* bmask = w.mask;  // explicit masks were staged there too
  // ---- fc3 -> log_softmax / CE (GT rows) -> D conv1 for the GT and noGT rows;
  //      D input rows are [lsm_gt; lsm_nogt; lsm_nogt] (:472, :492, :499) -----
  PC_TRY(launch_head_fwd(w.h2, G + PCADV_G_FC3_W, G + PCADV_G_FC3_B, a->labels, B, a->lambda_cls,
                         logits, w.dlogits, w.din, D + PCADV_D_CONV1_W, D + PCADV_D_CONV1_B, w.d1,
                         w.lpart, s));
  // ---- discriminator conv2, conv3 over the R = 3B rows (:499, :530, :546) ---
  PC_TRY(launch_linear_fwd(w.d1, D + PCADV_D_CONV2_W, D + PCADV_D_CONV2_B, w.d2, R, 256, 512,
                           PCADV_ACT_LRELU, nullptr, nullptr, 0, 0.f, s));
  PC_TRY(launch_linear_fwd(w.d2, D + PCADV_D_CONV3_W, D + PCADV_D_CONV3_B, w.d3, R, 256, 256,
                           PCADV_ACT_LRELU, nullptr, nullptr, 0, 0.f, s));
  // ---- conv4 -> conv5 -> fc, the three BCE terms, and back to dL/d(conv3) ---
  PC_TRY(launch_disc_tail(w.d3, B, D + PCADV_D_CONV4_W, D + PCADV_D_CONV4_B, D + PCADV_D_CONV5_W,
                          D + PCADV_D_CONV5_B, D + PCADV_D_FC_W, D + PCADV_D_FC_B, a->soft_gt,
                          a->soft_nogt, st, a->rng_seed, a->lambda_adv, w.dd3, w.dslabs, w.lpart3,
                          w.dout, s, w.gidx, C, N, ext ? nullptr : w.sortrec, w.z4, w.z5, w.a4,
                          rr * B));
  // ---- discriminator backward: parameter grads from rows [0,2B) (D loss),
  //      input grads of all rows (rows [2B,3B) feed the generator, D frozen).
  //      Every data gradient is stored as the layer below's dz (its activation
  //      derivative, and fc2's dropout, applied by the producer), so each
  //      backward launch reads dz as is: dd3 (k_disc_tail) -> dd2 -> dd1 ->
  //      (k_head_bwd) dh2 -> dh1 -> dgmax (raw: the max-pool has no activation)
  const int MW = 2 * B;
  {
    // + conv4's and conv5's weight gradients (block jobs over k_disc_tail's
    // z4 / z5 / a4 rows and the conv3 output) and the fc slabs' sum
    LinBwdExtra ex{};
    ex.job[0] = LinBwdJob{w.z4, w.d3, gD + PCADV_D_CONV4_W, gD + PCADV_D_CONV4_B, MW, 64, 256};
    ex.job[1] = LinBwdJob{w.z5, w.a4, gD + PCADV_D_CONV5_W, gD + PCADV_D_CONV5_B, MW, 64, 64};
    ex.njobs = 2;
    ex.red_src = w.dslabs;
    ex.red_dst = gD + PCADV_D_FC_W;
    ex.red_n = disc_tail_slab_n();
    ex.red_ld = (int)disc_tail_slab_floats();
    ex.red_cnt = disc_rowblocks(B);
    ex.dx_act = PCADV_ACT_LRELU;  // x = conv2 output
    PC_TRY(launch_linear_bwd(w.dd3, nullptr, PCADV_ACT_NONE, nullptr, nullptr, 0, 0.f, w.d2,
                             D + PCADV_D_CONV3_W, w.dd2, gD + PCADV_D_CONV3_W,
                             gD + PCADV_D_CONV3_B, R, MW, 256, 256, s, &ex));
  }
  // the adversarial rows' dd1 tiles also multiply into D conv1's weight: the
  // partials of its input gradient (summed by k_head_bwd), when the rows [2B, 3B)
  // start a row tile
  const bool chain = (2 * B) % 16 == 0;
  {
    LinBwdExtra ex{};
    ex.dx_act = PCADV_ACT_LRELU;  // x = conv1 output
    if (chain) {
      ex.chain_w = D + PCADV_D_CONV1_W;  // [512][40]
      ex.chain_out = w.ddp;
      ex.chain_row0 = 2 * B;
      ex.chain_n = 40;
    }
    PC_TRY(launch_linear_bwd(w.dd2, nullptr, PCADV_ACT_NONE, nullptr, nullptr, 0, 0.f, w.d1,
                             D + PCADV_D_CONV2_W, w.dd1, gD + PCADV_D_CONV2_W,
                             gD + PCADV_D_CONV2_B, R, MW, 256, 512, s, &ex));
  }
  // ---- D conv1 input grad of the adversarial rows -> log_softmax backward ->
  //      fc3 input grad (stored as fc2's dz); D conv1 weight grad; the losses -
  PC_TRY(launch_head_bwd(w.dd1, w.h2, bmask, a->drop_p, w.din, B, D + PCADV_D_CONV1_W,
                         G + PCADV_G_FC3_W, w.dlogits, w.dh2, nullptr, nullptr, w.lpart,
                         w.lpart3, a->losses, a->semi, a->lambda_semi, a->semi_th, logits,
                         w.dout, s, chain ? w.ddp : nullptr));
  // ---- generator head backward (:520); fc3's weight grad rides along -------
  {
    LinBwdExtra ex{};
    ex.job[0] = LinBwdJob{w.dlogits, w.h2, gG + PCADV_G_FC3_W, gG + PCADV_G_FC3_B, C, 40, 256};
    // D conv1's weight gradient over the D-loss rows: dz = conv1's dz (D conv2's
    // backward output), x = the D input rows
    ex.job[1] = LinBwdJob{w.dd1, w.din, gD + PCADV_D_CONV1_W, gD + PCADV_D_CONV1_B, 2 * B, 512, 40};
    ex.njobs = 2;
    ex.dx_act = PCADV_ACT_RELU;  // x = fc1 output
    PC_TRY(launch_linear_bwd(w.dh2, nullptr, PCADV_ACT_NONE, nullptr, nullptr, 0, 0.f, w.h1,
                             G + PCADV_G_FC2_W, w.dh1, gG + PCADV_G_FC2_W, gG + PCADV_G_FC2_B, C,
                             C, 256, 512, s, &ex));
  }
  {
    // fc2, fc3 and D are final: their Adam (optimizer.step / optimizer_D.step,
    // :558-559) rides along fc1's backward
    LinBwdExtra ex{};
    if (a->apply_adam && PCADV_EARLY_ADAM) {
      PC_REQUIRE(a->g_m && a->g_v && a->d_param && a->d_m && a->d_v, "adv_step: Adam buffers");
      ex.adam = fused_adam(a, true, true);
    }
    PC_TRY(launch_linear_bwd(w.dh1, nullptr, PCADV_ACT_NONE, nullptr, nullptr, 0, 0.f, gmax,
                             G + PCADV_G_FC1_W, dgmax, gG + PCADV_G_FC1_W, gG + PCADV_G_FC1_B, C,
                             C, 512, 1024, s, &ex));
  }
  return PCADV_OK;
}

// run_training_pointnet_cls's iteration (utils/trainer.py:222-268,
// feature_transform=False; BASELINE configs[1]): PointNetCls on B labelled
// clouds, loss = lambda_cls * CE, backward, Adam on the generator only.  The
// same kernels as the adversarial step minus the discriminator: the feature
// forward over C = B clouds, fc1, fc2 + dropout, fc3 + the CE + fc3's input
// gradient (k_cls_head), the head backward (k_linear_bwd x2), the sparse
// feature backward and one Adam launch.
static int cls_step(const pcadv_adv_args* a, hipStream_t s) {
  PC_REQUIRE(a && a->B > 0 && a->B <= 256 && a->N > 0 && a->pts_gt && a->labels && a->g_param &&
                 a->g_grad && a->step_count && a->losses,
             "cls_step: bad arguments");
  const int B = a->B, N = a->N, C = B;
  PC_REQUIRE(a->workspace && a->workspace_bytes >= carve(B, N, nullptr).total,
             "cls_step: workspace too small (need %zu bytes)", carve(B, N, nullptr).total);
  StepWs w = carve(B, N, static_cast<char*>(a->workspace));
  const float* G = a->g_param;
  float* gG = a->g_grad;
  const int32_t* st = a->step_count;
  float* logits = a->logits ? a->logits : w.logits;
  // part 3 (ABI 9): the head on a caller's pooled features (the feature-
  // transform generator's extractor runs outside, as adv_step's part 3):
  // fc1 .. the CE and back to dL/dgmax, no feature launches, no Adam
  PC_REQUIRE(a->part == 0 || a->part == 3, "cls_step: part %d (0 whole, 3 head on given features)",
             a->part);
  const bool ext = a->part == 3;
  PC_REQUIRE(!ext || (a->feat_gmax && a->feat_dgmax && !a->apply_adam && !a->ngather &&
                      !a->epi_ncounters && !a->epi_ring),
             "cls_step: part 3 needs feat_gmax / feat_dgmax and takes no Adam, gather or epilogue");
  const float* gmax = ext ? a->feat_gmax : w.gmax;
  float* dgmax = ext ? a->feat_dgmax : w.dgmax;
  const float* mask = nullptr;
  if (a->drop_mask_gt) {
    if (hipMemcpyAsync(w.mask, a->drop_mask_gt, sizeof(float) * B * 256, hipMemcpyDeviceToDevice,
                       s) != hipSuccess) {
      set_error("cls_step: mask staging copy failed");
      return PCADV_EHIP;
    }
    mask = w.mask;
  }
  const int32_t* rstep = mask ? nullptr : st;
  const int W = a->rng_world > 1 ? a->rng_world : 1, rr = W > 1 ? a->rng_rank : 0;
  PC_REQUIRE(rr >= 0 && rr < W, "cls_step: rng_rank %d not in [0, %d)", a->rng_rank, W);
  PC_TRY(check_folded_gather(a));
  if (!ext)
    PC_TRY(launch_feat_fwd_fused(a->pts_gt, a->pts_gt, B, C, N, G + PCADV_G_CONV1_W,
                                 G + PCADV_G_CONV1_B, G + PCADV_G_CONV2_W, G + PCADV_G_CONV2_B,
                                 G + PCADV_G_CONV3_W, G + PCADV_G_CONV3_B, G + PCADV_G_CONV4_W,
                                 G + PCADV_G_CONV4_B, w.x3, w.gmax, w.gidx, a->step_count,
                                 w.feat_ws, w.feat_ws_bytes, s, nullptr, a->precision, a->gather,
                                 a->ngather));
  PC_TRY(launch_linear_fwd(gmax, G + PCADV_G_FC1_W, G + PCADV_G_FC1_B, w.h1, C, 512, 1024,
                           PCADV_ACT_RELU, nullptr, nullptr, 0, 0.f, s));
  PC_TRY(launch_linear_fwd(w.h1, G + PCADV_G_FC2_W, G + PCADV_G_FC2_B, w.h2, C, 256, 512,
                           PCADV_ACT_RELU, mask, rstep, a->rng_seed, a->drop_p, s, 0,
                           mask ? nullptr : w.mask, B, rr * B, rr * B));
  // fc3, CrossEntropyLoss (train_classification.py:199), lambda_cls * dCE/dlogits
  // and fc3's input gradient, stored as fc2's dz (k_cls_head)
  PC_TRY(launch_cls_head(w.h2, w.mask, a->drop_p, G + PCADV_G_FC3_W, G + PCADV_G_FC3_B, a->labels,
                         B, a->lambda_cls, logits, w.dlogits, w.dh2, w.rowloss, s,
                         ext ? nullptr : w.gidx, C, N, ext || !PCADV_CLS_PRESORT ? nullptr : w.sortrec));
  {
    // fc2's backward; fc3's weight gradient and the CE batch mean ride along
    LinBwdExtra ex{};
    ex.job[0] = LinBwdJob{w.dlogits, w.h2, gG + PCADV_G_FC3_W, gG + PCADV_G_FC3_B, C, 40, 256};
    ex.njobs = 1;
    ex.red_src = w.rowloss;
    ex.red_dst = a->losses;
    ex.red_n = 1;
    ex.red_cnt = B;
    ex.red_ld = 1;
    ex.dx_act = PCADV_ACT_RELU;  // x = fc1 output
    PC_TRY(launch_linear_bwd(w.dh2, nullptr, PCADV_ACT_NONE, nullptr, nullptr, 0, 0.f, w.h1,
                             G + PCADV_G_FC2_W, w.dh1, gG + PCADV_G_FC2_W, gG + PCADV_G_FC2_B, C,
                             C, 256, 512, s, &ex));
  }
  {
    LinBwdExtra ex{};  // fc2 and fc3 are final: their Adam rides along fc1's backward
    if (a->apply_adam && !ext && PCADV_EARLY_ADAM) {
      PC_REQUIRE(a->g_m && a->g_v, "cls_step: Adam moments");
      ex.adam = fused_adam(a, false, true);
    }
    PC_TRY(launch_linear_bwd(w.dh1, nullptr, PCADV_ACT_NONE, nullptr, nullptr, 0, 0.f, gmax,
                             G + PCADV_G_FC1_W, dgmax, gG + PCADV_G_FC1_W, gG + PCADV_G_FC1_B, C,
                             C, 512, 1024, s, &ex));
  }
  if (ext) return PCADV_OK;
  // feature backward; Adam (generator only) fused into its finishing launch
  PC_REQUIRE(!a->apply_adam || (a->g_m && a->g_v), "cls_step: Adam moments");
  const FinAdam fa = fused_adam(a, false);
  IterEpi epi;
  bool epi_on;
  PC_TRY(step_epilogue(a, &epi, &epi_on));
  return launch_feat_bwd(w.dgmax, w.gidx, a->pts_gt, a->pts_gt, B, C, N, G + PCADV_G_CONV1_W,
                         G + PCADV_G_CONV1_B, G + PCADV_G_CONV2_W, G + PCADV_G_CONV2_B,
                         G + PCADV_G_CONV3_W, G + PCADV_G_CONV4_W, w.x3,
                         gG + PCADV_G_CONV1_W, gG + PCADV_G_CONV1_B, gG + PCADV_G_CONV2_W,
                         gG + PCADV_G_CONV2_B, gG + PCADV_G_CONV3_W, gG + PCADV_G_CONV3_B,
                         gG + PCADV_G_CONV4_W, gG + PCADV_G_CONV4_B, w.feat_ws, w.feat_ws_bytes,
                         s, nullptr, a->apply_adam ? &fa : nullptr,
                         PCADV_CLS_PRESORT ? w.sortrec : nullptr, epi_on ? &epi : nullptr,
                         a->precision == 1);
}

}  // namespace pcadv

using namespace pcadv;

extern "C" {

const char* pcadv_last_error(void) { return g_err; }
int pcadv_abi_version(void) { return 10; }

size_t pcadv_feat_fwd_workspace_bytes(int C, int N) { return feat_fwd_workspace_bytes(C, N); }

int pcadv_feat_fwd(const float* pts, int C, int N, const float* w1, const float* b1,
                   const float* w2, const float* b2, const float* w3, const float* b3,
                   const float* w4, const float* b4, float* x3, float* gmax, int32_t* gidx,
                   void* workspace, size_t workspace_bytes, hipStream_t stream) {
  return launch_feat_fwd_fused(pts, pts, C, C, N, w1, b1, w2, b2, w3, b3, w4, b4, x3, gmax, gidx,
                               nullptr, workspace, workspace_bytes, stream);
}

int pcadv_conv4_max(const void* x3, int C, int N, const float* w4, const float* b4, float* gmax,
                    int32_t* gidx, int precision, hipStream_t stream) {
  return launch_conv4_max(static_cast<const float*>(x3), C, N, w4, b4, gmax, gidx, stream,
                          precision);
}

int pcadv_feat_fwd_bf16(const float* pts, int C, int N, const float* w1, const float* b1,
                        const float* w2, const float* b2, const float* w3, const float* b3,
                        const float* w4, const float* b4, void* x3, float* gmax, int32_t* gidx,
                        void* workspace, size_t workspace_bytes, hipStream_t stream) {
  // x3: bf16 [C][N][128] (k_point_mlp<1>'s store)
  return launch_feat_fwd_fused(pts, pts, C, C, N, w1, b1, w2, b2, w3, b3, w4, b4,
                               static_cast<float*>(x3), gmax, gidx, nullptr, workspace,
                               workspace_bytes, stream, nullptr, 1);
}

#ifdef PCADV_STAMPS
// diagnostic build only: pcadv_feat_fwd with per-workgroup phase timestamps
int pcadv_feat_fwd_stamped(const float* pts, int C, int N, const float* w1, const float* b1,
                           const float* w2, const float* b2, const float* w3, const float* b3,
                           const float* w4, const float* b4, float* x3, float* gmax,
                           int32_t* gidx, void* workspace, size_t workspace_bytes,
                           uint64_t* stamps, hipStream_t stream) {
  return launch_feat_fwd_fused(pts, pts, C, C, N, w1, b1, w2, b2, w3, b3, w4, b4, x3, gmax, gidx,
                               nullptr, workspace, workspace_bytes, stream, stamps);
}
#endif

size_t pcadv_feat_bwd_workspace_bytes(int C, int N) { return feat_bwd_workspace_bytes(C, N); }

#if defined(PCADV_C4_CERT) && PCADV_C4_CERT
// diagnostic build only (tools/cert_diag.py): k_conv4_max's certification
// counters since the last read: [flagged at the rigorous bound, channels,
// flagged at 2^-17 x the bound, launches]
int pcadv_c4_cert_read(unsigned* host) { return c4_cert_read(host); }
#endif
#ifdef PCADV_STAMPS
int pcadv_tail_stamps(uint64_t* host) { return tail_stamps_read(host); }
int pcadv_chunk_stamps(uint64_t* host) { return chunk_stamps_read(host); }
int pcadv_lin_stamps(uint64_t* host, int reset) { return lin_stamps_read(host, reset); }

// diagnostic build only: pcadv_feat_bwd with per-workgroup phase timestamps
int pcadv_feat_bwd_stamped(const float* dgmax, const int32_t* gidx, const float* pts, int C,
                           int N, const float* w1, const float* b1, const float* w2,
                           const float* b2, const float* w3, const float* w4, const float* x3,
                           float* dw1, float* db1, float* dw2, float* db2, float* dw3, float* db3,
                           float* dw4, float* db4, void* workspace, size_t workspace_bytes,
                           uint64_t* stamps, hipStream_t stream) {
  return launch_feat_bwd(dgmax, gidx, pts, pts, C, C, N, w1, b1, w2, b2, w3, w4, x3, dw1, db1,
                         dw2, db2, dw3, db3, dw4, db4, workspace, workspace_bytes, stream, stamps);
}
#endif

int pcadv_feat_bwd(const float* dgmax, const int32_t* gidx, const float* pts, int C, int N,
                   const float* w1, const float* b1, const float* w2, const float* b2,
                   const float* w3, const float* w4, const float* x3, float* dw1, float* db1,
                   float* dw2, float* db2, float* dw3, float* db3, float* dw4, float* db4,
                   void* workspace, size_t workspace_bytes, hipStream_t stream) {
  PC_REQUIRE(C > 0 && N > 0, "feat_bwd: bad shape C=%d N=%d", C, N);
  return launch_feat_bwd(dgmax, gidx, pts, pts, C, C, N, w1, b1, w2, b2, w3, w4, x3, dw1, db1,
                         dw2, db2, dw3, db3, dw4, db4, workspace, workspace_bytes, stream);
}

int pcadv_conv_max_fwd(const float* x, int C, int N, int K, const float* w, const float* b, int O,
                       int relu_before_max, float* gmax, int32_t* gidx, hipStream_t stream) {
  PC_REQUIRE(K == 128, "conv_max_fwd: only K=128 is implemented (got %d)", K);
  PC_REQUIRE(C > 0 && N > 0 && O > 0 && O % 128 == 0, "conv_max_fwd: bad shape C=%d N=%d O=%d", C,
             N, O);
  return launch_conv_max128(x, C, N, w, b, O, relu_before_max != 0, gmax, gidx, stream);
}

int pcadv_linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int Nout,
                     int K, int act, const float* drop_mask, const int32_t* rng_step,
                     uint64_t rng_seed, float drop_p, int add_identity_k, hipStream_t stream) {
  return launch_linear_fwd(x, w, b, y, M, Nout, K, act, drop_mask, rng_step, rng_seed, drop_p,
                           stream, add_identity_k);
}

int pcadv_pw_fwd(const float* x, int M, int K, const float* w, const float* b, int O, int act,
                 int w_kmajor, int rows_per_w, float* y, hipStream_t stream) {
  return launch_pw_fwd(x, M, K, w, b, O, act, w_kmajor, rows_per_w, y, stream);
}

int pcadv_pw_chain(const float* x, int M, int K, const pcadv_pw_layer* layers, int n,
                   hipStream_t stream) {
  return launch_pw_chain(x, M, K, layers, n, stream);
}

int pcadv_pw_bwd_data(const float* dy, const float* y, int act, int M, int O, const float* w,
                      int K, int w_kmajor, int rows_per_w, float* dx, int accumulate,
                      hipStream_t stream) {
  return launch_pw_bwd_data(dy, y, act, M, O, w, K, w_kmajor, rows_per_w, dx, accumulate, stream);
}

size_t pcadv_pw_bwd_weight_workspace_bytes(int M, int O, int K) {
  return pw_bwd_weight_workspace_bytes(M, O, K);
}

int pcadv_pw_bwd_weight(const float* dy, const float* y, int act, const float* x, int M, int O,
                        int K, int rows_per_group, int dw_kmajor, float* dw, float* db,
                        void* workspace, size_t workspace_bytes, hipStream_t stream) {
  return launch_pw_bwd_weight(dy, y, act, x, M, O, K, rows_per_group, dw_kmajor, dw, db,
                              workspace, workspace_bytes, stream);
}

int pcadv_pw_wgrad_finish(const pcadv_pw_wgrad_job* jobs, int njobs, hipStream_t stream) {
  return launch_pw_wgrad_finish(jobs, njobs, stream);
}

int pcadv_conv_max_bwd(const float* dgmax, const int32_t* gidx, const float* gmax_relu,
                       const float* x, int C, int N, int K, const float* w, int O, float* dw,
                       float* db, float* dx, int dx_relu, hipStream_t stream) {
  return launch_convmax_bwd(dgmax, gidx, gmax_relu, x, C, N, K, w, O, dw, db, dx, stream,
                            dx_relu);
}

int pcadv_tnet_reg_fwd(const float* T, int B, int k, float* norms, float* reg,
                       hipStream_t stream) {
  PC_REQUIRE(norms && reg, "tnet_reg_fwd: norms and reg are required");
  return launch_tnet_reg(T, B, k, norms, reg, nullptr, nullptr, stream);
}

int pcadv_tnet_reg_bwd(const float* T, int B, int k, const float* grad_reg, float* dT,
                       hipStream_t stream) {
  PC_REQUIRE(grad_reg && dT, "tnet_reg_bwd: grad_reg and dT are required");
  return launch_tnet_reg(T, B, k, nullptr, nullptr, grad_reg, dT, stream);
}

int pcadv_tnet_reg_step(const float* T, int B, int k, float* norms, float* reg,
                        const float* grad_reg, float* dT, int32_t* step_count,
                        hipStream_t stream) {
  PC_REQUIRE(norms && reg && grad_reg && dT, "tnet_reg_step: norms, reg, grad_reg and dT are required");
  return launch_tnet_reg(T, B, k, norms, reg, grad_reg, dT, stream, 1, step_count);
}

int pcadv_linear_bwd(const float* dy, const float* y, int act, const float* drop_mask,
                     const int32_t* rng_step, uint64_t rng_seed, float drop_p, const float* x,
                     const float* w, float* dx, float* dw, float* db, int M, int m_w, int Nout,
                     int K, hipStream_t stream) {
  return launch_linear_bwd(dy, y, act, drop_mask, rng_step, rng_seed, drop_p, x, w, dx, dw, db, M,
                           m_w, Nout, K, stream);
}

int pcadv_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
               int32_t* step_count, float lr, float beta1, float beta2, float eps,
               hipStream_t stream) {
  PC_REQUIRE(n > 0 && step_count, "adam: bad arguments");
  PC_TRY(launch_adam2(param, grad, exp_avg, exp_avg_sq, n, lr, nullptr, nullptr, nullptr, nullptr,
                      0, 0.f, step_count, 1, beta1, beta2, eps, stream));
  return launch_inc(step_count, stream);
}

int pcadv_concat2(const float* a, int64_t na, const float* b, int64_t nb, float* out,
                  int32_t* inc_counter, hipStream_t stream) {
  return launch_concat2(a, na, b, nb, out, inc_counter, stream);
}

int pcadv_adam2(float* p0, const float* g0, float* m0, float* v0, int64_t n0, float lr0,
                float* p1, const float* g1, float* m1, float* v1, int64_t n1, float lr1,
                const int32_t* step_count, float beta1, float beta2, float eps,
                hipStream_t stream) {
  PC_REQUIRE(n0 > 0 && n1 >= 0 && step_count && p0 && g0 && m0 && v0 &&
                 (n1 == 0 || (p1 && g1 && m1 && v1)),
             "adam2: bad arguments");
  return launch_adam2(p0, g0, m0, v0, n0, lr0, p1, g1, m1, v1, n1, lr1, step_count, 0, beta1,
                      beta2, eps, stream);
}

// ---- dense point-wise GEMM engine (segmentation net) -----------------------
int pcadv_gemm(const float* a, int64_t lda, int ta, const float* b, int64_t ldb, int tb,
               float* c, int64_t ldc, int M, int N, int K, const float* bias,
               const float* bias_rows, int rows_per_group, int relu, int accumulate,
               const float* cmask, int64_t ldm, int precise, void* c_hi, void* c_lo, int64_t ldcp,
               hipStream_t stream) {
  return launch_gemm(a, lda, ta, b, ldb, tb, c, ldc, M, N, K, bias, bias_rows, rows_per_group,
                     relu, accumulate, cmask, ldm, precise, c_hi, c_lo, ldcp, stream);
}

int pcadv_gemm_bf2(const void* a_hi, const void* a_lo, int64_t lda, const void* b_hi,
                   const void* b_lo, int64_t ldb, float* c, int64_t ldc, void* c_hi, void* c_lo,
                   int64_t ldcp, int M, int N, int K, const float* bias, const float* bias_rows,
                   int rows_per_group, int relu, int accumulate, const float* cmask, int64_t ldm,
                   hipStream_t stream) {
  return launch_gemm_bf2(a_hi, a_lo, lda, b_hi, b_lo, ldb, c, ldc, c_hi, c_lo, ldcp, M, N, K, bias,
                         bias_rows, rows_per_group, relu, accumulate, cmask, ldm, stream);
}

int pcadv_split_bf2(const float* x, int64_t ld, int rows, int cols, void* hi, void* lo,
                    int64_t ldo, hipStream_t stream) {
  return launch_split_bf2(x, ld, rows, cols, hi, lo, ldo, stream);
}

int pcadv_split_bf3(const float* x, int64_t ld, int rows, int cols, void* hi, void* mid, void* lo,
                    int64_t ldo, hipStream_t stream) {
  return launch_split_bf3(x, ld, rows, cols, hi, mid, lo, ldo, stream);
}

int pcadv_gemm_b3(const float* a, int64_t lda, const void* b_hi, const void* b_mid,
                  const void* b_lo, int64_t ldb, float* c, int64_t ldc, int M, int N, int K,
                  const float* bias, const float* bias_rows, int rows_per_group, int relu,
                  int accumulate, hipStream_t stream) {
  return launch_gemm_b3(a, lda, b_hi, b_mid, b_lo, ldb, c, ldc, M, N, K, bias, bias_rows,
                        rows_per_group, relu, accumulate, stream);
}

size_t pcadv_gemm_wgrad_workspace_bytes(int rows, int O, int Kin, int rows_per_group) {
  return gemm_wgrad_workspace_bytes(rows, O, Kin, rows_per_group);
}

int pcadv_gemm_wgrad(const float* dz, int64_t ldz, const float* x, int64_t ldx, int rows, int O,
                     int Kin, float* dw, int64_t ldo, float* db, float* gsum, int rows_per_group,
                     int accumulate, void* workspace, size_t workspace_bytes, hipStream_t stream) {
  return launch_gemm_wgrad(dz, ldz, x, ldx, rows, O, Kin, dw, ldo, db, gsum, rows_per_group,
                           accumulate, workspace, workspace_bytes, stream);
}

int pcadv_gemm_wgrad_slabs(const pcadv_wgrad_desc* w, const pcadv_gemm_desc* g,
                           hipStream_t stream) {
  return launch_gemm_wgrad_slabs(w, g, stream);
}

int pcadv_wgrad_finish(const pcadv_wgrad_desc* w, int n, hipStream_t stream) {
  return launch_wgrad_finish(w, n, stream);
}

int pcadv_wgrad_small(const float* s, int64_t lds, int B, int O, const float* x0, int64_t ldx0,
                      int K0, float* dw0, const float* x1, int64_t ldx1, int K1, float* dw1,
                      int64_t ldo, int accumulate, hipStream_t stream) {
  return launch_wgrad_small(s, lds, B, O, x0, ldx0, K0, dw0, x1, ldx1, K1, dw1, ldo, accumulate,
                            stream);
}

size_t pcadv_colsum_workspace_bytes(int M, int N) { return colsum_workspace_bytes(M, N); }

int pcadv_colsum(const float* x, const float* ymask, int64_t ld, int64_t ldm, int M, int N,
                 float* out, int accumulate, void* workspace, size_t workspace_bytes,
                 hipStream_t stream) {
  return launch_colsum(x, ymask, ld, ldm, M, N, out, accumulate, workspace, workspace_bytes,
                       stream);
}

int pcadv_group_colsum(const float* x, const float* ymask, int64_t ld, int64_t ldm, int M, int N,
                       int rows_per_group, float* out, hipStream_t stream) {
  return launch_group_colsum(x, ymask, ld, ldm, M, N, rows_per_group, out, stream);
}

size_t pcadv_conv_max_x3_workspace_bytes(int C, int Npts, int O) {
  return conv_max_x3_workspace_bytes(C, Npts, O);
}

int pcadv_conv_max_x3(const float* x, int64_t ldx, int C, int Npts, int K, const float* w,
                      const float* b, int O, int relu, float* gmax, int32_t* gidx,
                      void* workspace, size_t workspace_bytes, hipStream_t stream) {
  return launch_conv_max_x3(x, ldx, C, Npts, K, w, b, O, relu, gmax, gidx, workspace,
                            workspace_bytes, stream, nullptr, nullptr, 0, nullptr, nullptr);
}

int pcadv_conv_max_bf2(const float* x, int64_t ldx, const void* x_hi, const void* x_lo,
                       int64_t ldxp, int C, int Npts, int K, const float* w, const void* w_hi,
                       const void* w_lo, const float* b, int O, int relu, float* gmax,
                       int32_t* gidx, void* workspace, size_t workspace_bytes,
                       hipStream_t stream) {
  PC_REQUIRE(x_hi && x_lo && w_hi && w_lo, "conv_max_bf2: planes required");
  return launch_conv_max_x3(x, ldx, C, Npts, K, w, b, O, relu, gmax, gidx, workspace,
                            workspace_bytes, stream, x_hi, x_lo, ldxp, w_hi, w_lo);
}

int pcadv_conv_max_x3_bwd(const float* dgmax, const float* gmax, const int32_t* gidx,
                          const float* x, int64_t ldx, int C, int Npts, int O, int K,
                          const float* w, float* dw, float* db, float* dx, int64_t lddx,
                          int relu_x, hipStream_t stream) {
  return launch_cmx_bwd(dgmax, gmax, gidx, x, ldx, C, Npts, O, K, w, dw, db, dx, lddx, relu_x,
                        stream);
}

int pcadv_gather_clouds(const float* src, int64_t n_src, int npts, int src_npts,
                        const int64_t* idx, int B, const int64_t* src_lab, int lab_width,
                        const int64_t* src_seg, double sigma, double clip, const double* noise,
                        uint64_t seed, const int32_t* step, float* out, int64_t* out_lab,
                        int64_t* out_seg, int64_t rng_row0, hipStream_t stream) {
  return launch_gather_clouds(src, n_src, npts, src_npts, idx, B, src_lab, lab_width, src_seg,
                              sigma, clip, noise, seed, step, out, out_lab, out_seg, stream,
                              nullptr, rng_row0);
}

int pcadv_gather_clouds_at(const float* src, int64_t n_src, int npts, int src_npts,
                           const int64_t* order, const int32_t* cursor, int B,
                           const int64_t* src_lab, int lab_width, const int64_t* src_seg,
                           double sigma, double clip, uint64_t seed, const int32_t* step,
                           float* out, int64_t* out_lab, int64_t* out_seg, int64_t rng_row0,
                           hipStream_t stream) {
  PC_REQUIRE(cursor, "gather_clouds_at: cursor required");
  return launch_gather_clouds(src, n_src, npts, src_npts, order, B, src_lab, lab_width, src_seg,
                              sigma, clip, nullptr, seed, step, out, out_lab, out_seg, stream,
                              cursor, rng_row0);
}

int pcadv_gather_clouds_multi(const pcadv_gather_job* jobs, int njobs, hipStream_t stream) {
  return launch_gather_multi(jobs, njobs, stream);
}

int pcadv_iter_epilogue(int32_t* counters, int ncounters, const float* losses, int nl,
                        float* ring, int slots, int32_t* ring_count, hipStream_t stream) {
  return launch_iter_epilogue(counters, ncounters, losses, nl, ring, slots, ring_count, stream);
}

size_t pcadv_row_ce_workspace_bytes(int M) { return row_ce_workspace_bytes(M); }

int pcadv_row_ce(const float* logits, int64_t ld, const int64_t* labels, int M, int ncls,
                 float scale, float* loss, float* dlogits, void* workspace,
                 size_t workspace_bytes, hipStream_t stream) {
  return launch_row_ce(logits, ld, labels, M, ncls, scale, loss, dlogits, workspace,
                       workspace_bytes, stream);
}

size_t pcadv_adv_step_workspace_bytes(int B, int N) { return carve(B, N, nullptr).total; }

int pcadv_adv_step(const pcadv_adv_args* args, hipStream_t stream) { return adv_step(args, stream); }

int pcadv_adv_step_adam(const pcadv_adv_args* args, hipStream_t stream) {
  return adv_adam(args, stream);
}

int pcadv_cls_step(const pcadv_adv_args* args, hipStream_t stream) { return cls_step(args, stream); }

}  // extern "C"

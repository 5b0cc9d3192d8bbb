// Batch assembly on the device for the data path: the whole
// split stays resident in HBM and each batch is a gather of B clouds by index
// plus the reference's per-point jitter (dataset/modelNetData.py:80-91,
// jitter_point_cloud: data + clip(sigma * randn(N, 3), -clip, clip), applied in
// __getitem__ when data_augmentation is on, :73-78), the labels and part ids
// gathered alongside.  Replaces the host DataLoader + H2D copy per step.
//
// One thread per point (3 floats), coalesced along the point axis.  Noise:
// explicit f64 standard-normal draws (parity with numpy, which jitters in f64
// and rounds to f32 in __getitem__), or Philox-4x32 draws keyed by (seed,
// device step counter, RNG_JITTER, point) turned into normals by Box-Muller, so
// a captured graph jitters differently on every replay.
#include "common.h"

namespace pcadv {


// One batch point t of a gather (below): batch row b = t / npts, point p.
__device__ __forceinline__ void gather_point(
    int64_t t, const float* __restrict__ src, int64_t n_src, int npts, int src_npts,
    const int64_t* __restrict__ idx, int B, const int64_t* __restrict__ src_lab, int lab_width,
    const int64_t* __restrict__ src_seg, double sigma_d, double clip_d,
    const double* __restrict__ noise, uint64_t seed, const int32_t* __restrict__ step,
    float* __restrict__ out, int64_t* __restrict__ out_lab, int64_t* __restrict__ out_seg,
    const int32_t* __restrict__ cursor, int64_t rng_row0) {
  if (t >= (int64_t)B * npts) return;
  const int b = (int)(t / npts), p = (int)(t % npts);
  // cursor: batch k = *cursor of an epoch order held in idx (a graph-fed loader)
  const int64_t c = idx[(cursor ? (int64_t)*cursor * B : 0) + b];
  // DeviceCloudLoader.gather() rejects out-of-range indices on the host before
  // the launch (its own epoch order is in range by construction); this guard
  // only keeps a bad index from reading outside the split
  if (c < 0 || c >= n_src) return;
  const float* s = src + ((size_t)c * src_npts + p) * 3;
  float* o = out + (size_t)t * 3;
  const float x0 = s[0], x1 = s[1], x2 = s[2];
  const float sigma = (float)sigma_d, clip = (float)clip_d;
  if (sigma_d > 0.0) {
    if (noise) {  // f64 like numpy (sigma, clip are Python floats there)
      const double* z = noise + (size_t)t * 3;
      const double sg = sigma_d, cl = clip_d;
      o[0] = (float)((double)x0 + fmin(fmax(sg * z[0], -cl), cl));
      o[1] = (float)((double)x1 + fmin(fmax(sg * z[1], -cl), cl));
      o[2] = (float)((double)x2 + fmin(fmax(sg * z[2], -cl), cl));
    } else {
      const uint32_t st = step ? (uint32_t)*step : 0u;
      // keyed by the point's row in the global batch (a data-parallel rank's
      // batch rows start at rng_row0), so W ranks jitter as one loader would
      const int64_t tg = t + rng_row0 * npts;
      o[0] = jitter_coord(x0, sigma, clip, jitter_normal(seed, st, tg, 0));
      o[1] = jitter_coord(x1, sigma, clip, jitter_normal(seed, st, tg, 1));
      o[2] = jitter_coord(x2, sigma, clip, jitter_normal(seed, st, tg, 2));
    }
  } else {
    o[0] = x0;
    o[1] = x1;
    o[2] = x2;
  }
  if (out_seg && src_seg) out_seg[t] = src_seg[(size_t)c * src_npts + p];
  if (p < lab_width && out_lab && src_lab) out_lab[(size_t)b * lab_width + p] = src_lab[(size_t)c * lab_width + p];
}

__global__ void __launch_bounds__(256)
k_gather_clouds(const float* __restrict__ src, int64_t n_src, int npts, int src_npts,
                const int64_t* __restrict__ idx, int B, const int64_t* __restrict__ src_lab,
                int lab_width, const int64_t* __restrict__ src_seg, double sigma_d, double clip_d,
                const double* __restrict__ noise, uint64_t seed, const int32_t* __restrict__ step,
                float* __restrict__ out, int64_t* __restrict__ out_lab,
                int64_t* __restrict__ out_seg, const int32_t* __restrict__ cursor, int64_t rng_row0) {
  gather_point((int64_t)blockIdx.x * 256 + threadIdx.x, src, n_src, npts, src_npts, idx, B, src_lab,
               lab_width, src_seg, sigma_d, clip_d, noise, seed, step, out, out_lab, out_seg,
               cursor, rng_row0);
}

// Several graph-fed loaders' batches in one launch (blockIdx.y = job): the
// iteration's GT and no-GT gathers without a launch boundary between them.
constexpr int GATHER_MAXJOBS = 4;
struct GatherJobs {
  pcadv_gather_job j[GATHER_MAXJOBS];
};
__global__ void __launch_bounds__(256) k_gather_multi(GatherJobs jobs) {
  const pcadv_gather_job& j = jobs.j[blockIdx.y];
  gather_point((int64_t)blockIdx.x * 256 + threadIdx.x, j.src, j.n_src, j.npts, j.src_npts,
               j.order, j.B, j.src_lab, j.lab_width, j.src_seg, j.sigma, j.clip, nullptr, j.seed,
               j.step, j.out, j.out_lab, j.out_seg, j.cursor, j.rng_row0);
}

int launch_gather_clouds(const float* src, int64_t n_src, int npts, int src_npts,
                         const int64_t* idx, int B, const int64_t* src_lab, int lab_width,
                         const int64_t* src_seg, double sigma, double clip, const double* noise,
                         uint64_t seed, const int32_t* step, float* out, int64_t* out_lab,
                         int64_t* out_seg, hipStream_t s, const int32_t* cursor, int64_t rng_row0) {
  PC_REQUIRE(src && idx && out && n_src > 0 && B > 0 && npts > 0 && src_npts >= npts,
             "gather_clouds: bad arguments (n_src=%lld B=%d npts=%d src_npts=%d)",
             (long long)n_src, B, npts, src_npts);
  PC_REQUIRE(sigma >= 0.0 && (sigma == 0.0 || clip > 0.0), "gather_clouds: clip must be > 0");
  PC_REQUIRE(!src_lab || (lab_width > 0 && lab_width <= npts && out_lab), "gather_clouds: labels");
  PC_REQUIRE(!src_seg || out_seg, "gather_clouds: part ids");
  const int64_t n = (int64_t)B * npts;
  hipLaunchKernelGGL(k_gather_clouds, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src,
                     n_src, npts, src_npts, idx, B, src_lab, lab_width, src_seg, sigma, clip, noise,
                     seed, step, out, out_lab, out_seg, cursor, rng_row0);
  PC_HIP_CHECK_LAUNCH("k_gather_clouds");
  return PCADV_OK;
}

// The end of a graph-replayed training iteration as a launch of its own
// (iter_epi_wave, common.h).  One wave.
__global__ void __launch_bounds__(64) k_iter_epilogue(IterEpi e) { iter_epi_wave(e, threadIdx.x); }

int check_iter_epi(const IterEpi& e) {
  PC_REQUIRE(e.ncounters >= 0 && e.ncounters <= 64 && (e.ncounters == 0 || e.counters),
             "iter_epilogue: %d counters (at most 64)", e.ncounters);
  PC_REQUIRE(!e.ring || (e.ring_count && e.losses && e.nl > 0 && e.nl <= 32 && e.slots > 0),
             "iter_epilogue: bad loss ring (nl=%d slots=%d)", e.nl, e.slots);
  return PCADV_OK;
}

int launch_iter_epilogue(int32_t* counters, int ncounters, const float* losses, int nl, float* ring,
                         int slots, int32_t* ring_count, hipStream_t s) {
  const IterEpi e{counters, ncounters, losses, nl, ring, slots, ring_count};
  const int rc = check_iter_epi(e);
  if (rc != PCADV_OK) return rc;
  hipLaunchKernelGGL(k_iter_epilogue, dim3(1), dim3(64), 0, s, e);
  PC_HIP_CHECK_LAUNCH("k_iter_epilogue");
  return PCADV_OK;
}

// out = [a; b] (f32 elements; 16-B pieces where both halves are 16-B aligned)
// and, with inc, *inc += 1 by one thread: the feature-transform step's first
// launch (its GT and no-GT batches as one 2B-cloud input, the iteration's step
// number advanced for the device draws and Adam).
__global__ void __launch_bounds__(256)
k_concat2(const float* __restrict__ a, int64_t na, const float* __restrict__ b, int64_t nb,
          float* __restrict__ out, int32_t* __restrict__ inc, int vec) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (inc && t == 0) *inc += 1;
  if (vec) {
    const int64_t qa = na / 4, q = qa + nb / 4;
    if (t < q)
      reinterpret_cast<f32x4*>(out)[t] =
          t < qa ? reinterpret_cast<const f32x4*>(a)[t] : reinterpret_cast<const f32x4*>(b)[t - qa];
    return;
  }
  if (t < na + nb) out[t] = t < na ? a[t] : b[t - na];
}

int launch_concat2(const float* a, int64_t na, const float* b, int64_t nb, float* out,
                   int32_t* inc, hipStream_t s) {
  PC_REQUIRE(a && b && out && na >= 0 && nb >= 0 && na + nb > 0, "concat2: bad arguments");
  const bool vec = na % 4 == 0 && nb % 4 == 0 && ((uintptr_t)a & 15) == 0 &&
                   ((uintptr_t)b & 15) == 0 && ((uintptr_t)out & 15) == 0;
  const int64_t n = vec ? (na + nb) / 4 : na + nb;
  hipLaunchKernelGGL(k_concat2, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, na, b, nb,
                     out, inc, vec ? 1 : 0);
  PC_HIP_CHECK_LAUNCH("k_concat2");
  return PCADV_OK;
}

int launch_gather_multi(const pcadv_gather_job* jobs, int njobs, hipStream_t s) {
  PC_REQUIRE(jobs && njobs >= 1 && njobs <= GATHER_MAXJOBS, "gather_multi: %d jobs (1..%d)", njobs,
             GATHER_MAXJOBS);
  GatherJobs g{};
  int64_t nmax = 0;
  for (int k = 0; k < njobs; ++k) {
    const pcadv_gather_job& j = jobs[k];
    PC_REQUIRE(j.src && j.order && j.cursor && j.out && j.n_src > 0 && j.B > 0 && j.npts > 0 &&
                   j.src_npts >= j.npts,
               "gather_multi: job %d: bad arguments (n_src=%lld B=%d npts=%d src_npts=%d)", k,
               (long long)j.n_src, j.B, j.npts, j.src_npts);
    PC_REQUIRE(j.sigma >= 0.0 && (j.sigma == 0.0 || j.clip > 0.0),
               "gather_multi: job %d: clip must be > 0", k);
    PC_REQUIRE(!j.src_lab || (j.lab_width > 0 && j.lab_width <= j.npts && j.out_lab),
               "gather_multi: job %d: labels", k);
    PC_REQUIRE(!j.src_seg || j.out_seg, "gather_multi: job %d: part ids", k);
    g.j[k] = j;
    const int64_t n = (int64_t)j.B * j.npts;
    if (n > nmax) nmax = n;
  }
  hipLaunchKernelGGL(k_gather_multi, dim3((unsigned)((nmax + 255) / 256), njobs), dim3(256), 0, s, g);
  PC_HIP_CHECK_LAUNCH("k_gather_multi");
  return PCADV_OK;
}

}  // namespace pcadv

// Optimizer of the adversarial step (gfx950): k_adam, torch.optim.Adam
// (single-tensor formula, train_classification.py:110-122) over flat buffers.
// The loss heads live in tail.hip.
#include "common.h"

namespace pcadv {

// torch.optim.Adam (adam_elem, common.h) over up to two segments (generator,
// discriminator) per launch.
struct AdamSeg {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  float lr;
};

__global__ void __launch_bounds__(256)
k_adam(AdamSeg s0, AdamSeg s1, int nblk0, const int32_t* __restrict__ step_count, int step_offset,
       float b1, float b2, float eps) {
  const bool first = (int)blockIdx.x < nblk0;
  const AdamSeg s = first ? s0 : s1;
  const int blk = first ? blockIdx.x : blockIdx.x - nblk0;
  const int nblk = first ? nblk0 : gridDim.x - nblk0;
  const AdamHp h = adam_hp(step_count, step_offset, b1, b2, eps, s.lr);
  const int64_t n4 = s.n / 4;
  for (int64_t i = (int64_t)blk * 256 + threadIdx.x; i < n4; i += (int64_t)nblk * 256) {
    const f32x4 p4 = reinterpret_cast<f32x4*>(s.p)[i];
    const f32x4 g4 = reinterpret_cast<const f32x4*>(s.g)[i];
    const f32x4 m4 = reinterpret_cast<f32x4*>(s.m)[i];
    const f32x4 v4 = reinterpret_cast<f32x4*>(s.v)[i];
    float p[4] = {p4.x, p4.y, p4.z, p4.w}, g[4] = {g4.x, g4.y, g4.z, g4.w};
    float m[4] = {m4.x, m4.y, m4.z, m4.w}, v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) adam_elem(p[e], g[e], m[e], v[e], h);
    reinterpret_cast<f32x4*>(s.p)[i] = f32x4{p[0], p[1], p[2], p[3]};
    reinterpret_cast<f32x4*>(s.m)[i] = f32x4{m[0], m[1], m[2], m[3]};
    reinterpret_cast<f32x4*>(s.v)[i] = f32x4{v[0], v[1], v[2], v[3]};
  }
  if (blk == 0 && threadIdx.x < (s.n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    adam_elem(s.p[i], s.g[i], s.m[i], s.v[i], h);
  }
}

__global__ void k_inc(int32_t* c) { *c += 1; }




static int adam_blocks(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  if (b > 1024) b = 1024;
  return (int)(b < 1 ? 1 : b);
}

// step_offset: 1 when *step_count still holds the completed-step count (the
// standalone pcadv_adam), 0 when the fused step already advanced it.
int launch_adam2(float* p0, const float* g0, float* m0, float* v0, int64_t n0, float lr0,
                 float* p1, const float* g1, float* m1, float* v1, int64_t n1, float lr1,
                 const int32_t* step_count, int step_offset, float b1, float b2, float eps,
                 hipStream_t s) {
  AdamSeg a{p0, g0, m0, v0, n0, lr0};
  AdamSeg b{p1, g1, m1, v1, n1, lr1};
  const int nb0 = adam_blocks(n0);
  const int nb1 = n1 > 0 ? adam_blocks(n1) : 0;
  hipLaunchKernelGGL(k_adam, dim3(nb0 + nb1), dim3(256), 0, s, a, b, nb0, step_count, step_offset,
                     b1, b2, eps);
  PC_HIP_CHECK_LAUNCH("k_adam");
  return PCADV_OK;
}

int launch_inc(int32_t* c, hipStream_t s) {
  hipLaunchKernelGGL(k_inc, dim3(1), dim3(1), 0, s, c);
  PC_HIP_CHECK_LAUNCH("k_inc");
  return PCADV_OK;
}

}  // namespace pcadv

// Loss heads and optimizer of the adversarial step (gfx950).
//
// k_cls_loss  : F.log_softmax of both generator batches (utils/trainer.py:472,492)
//               + CrossEntropyLoss on the GT batch (:469, train_classification.py:199),
//               writes the discriminator input rows [lsm_gt; lsm_nogt; lsm_nogt].
// k_disc_loss : BCEWithLogitsLoss terms (train_classification.py:200) of
//               trainer.py:507 (adv, label 1), :537 (D on GT, U(0.7,1.05) x 0.5)
//               and :553 (D on noGT, U(0,0.305) x 0.5); soft labels of
//               make_D_label(random=True) (utils/utils.py:22-31) drawn on device.
// k_lsm_bwd   : log_softmax backward of the noGT rows.
// k_adam      : torch.optim.Adam (single-tensor formula) over flat buffers.
#include "common.h"

namespace pcadv {

// One wave per row of K <= 64 logits.
__global__ void __launch_bounds__(1024)
k_cls_loss(const float* __restrict__ logits, const int64_t* __restrict__ labels, int B, int K,
           float lambda_cls, float* __restrict__ dinput, float* __restrict__ dlogits,
           float* __restrict__ losses) {
  __shared__ float row_loss[1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int m = wave; m < 2 * B; m += 16) {
    const float v = lane < K ? logits[(size_t)m * K + lane] : -INFINITY;
    float mx = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float e = lane < K ? expf(v - mx) : 0.f;
    float se = e;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const float lse = logf(se);
    const float lsm = (v - mx) - lse;
    if (lane < K) {
      dinput[(size_t)m * K + lane] = lsm;
      if (m >= B) dinput[(size_t)(m + B) * K + lane] = lsm;
    }
    if (m < B) {
      const int y = (int)labels[m];
      const float sm = expf(lsm);
      if (lane < K) dlogits[(size_t)m * K + lane] = lambda_cls * ((lane == y ? sm - 1.f : sm) / (float)B);
      const float ly = __shfl(lsm, y);
      if (lane == 0) row_loss[m] = -ly;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int m = 0; m < B; ++m) s += row_loss[m];
    losses[0] = s / (float)B;
  }
}

__device__ __forceinline__ float bce_logits(float x, float y) {
  return fmaxf(x, 0.f) - x * y + log1pf(expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// dout rows: [0,B) D(lsm_gt), [B,2B) D(lsm_nogt) for the D loss, [2B,3B) the
// same D(lsm_nogt) for the generator's adversarial loss.
__global__ void __launch_bounds__(256)
k_disc_loss(const float* __restrict__ dout, int B, const float* __restrict__ soft_gt,
            const float* __restrict__ soft_nogt, const int32_t* __restrict__ step, uint64_t seed,
            float lambda_adv, float* __restrict__ ddout, float* __restrict__ losses) {
  __shared__ float l[3][256];
  const int t = threadIdx.x;
  for (int m = t; m < 3 * B; m += 256) {
    const float x = dout[m];
    float y, f;
    int which;
    if (m < B) {
      y = soft_gt ? soft_gt[m]
                  : 0.7f + 0.35f * rng_uniform(seed, (uint32_t)*step, RNG_LABEL_GT, (uint32_t)m);
      f = 0.5f;
      which = 1;
    } else if (m < 2 * B) {
      y = soft_nogt ? soft_nogt[m - B]
                    : 0.305f * rng_uniform(seed, (uint32_t)*step, RNG_LABEL_NOGT, (uint32_t)(m - B));
      f = 0.5f;
      which = 2;
    } else {
      y = 1.f;
      f = lambda_adv;
      which = 0;
    }
    ddout[m] = f * (sigmoidf_(x) - y) / (float)B;
    l[which][m % B] = bce_logits(x, y);
  }
  __syncthreads();
  if (t < 3) {
    float s = 0.f;
    for (int m = 0; m < B; ++m) s += l[t][m];
    s /= (float)B;
    if (t == 0) losses[1] = s;
    else losses[1 + t] = 0.5f * s;
  }
}

// dlogits[m] = dlsm - softmax * sum(dlsm) for the noGT rows m in [B, 2B);
// lsm rows live at dinput[m], their gradient at ddinput[m + B].
__global__ void __launch_bounds__(1024)
k_lsm_bwd(const float* __restrict__ dinput, const float* __restrict__ ddinput, int B, int K,
          float* __restrict__ dlogits) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int m = B + wave; m < 2 * B; m += 16) {
    const float g = lane < K ? ddinput[(size_t)(m + B) * K + lane] : 0.f;
    float s = g;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane < K) dlogits[(size_t)m * K + lane] = g - expf(dinput[(size_t)m * K + lane]) * s;
  }
}

// torch.optim.Adam, single-tensor path:
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2)
//   p.addcdiv_(m, sqrt(v)/sqrt(1-b2^t) + eps, value=-lr/(1-b1^t))
// Up to two segments (generator, discriminator) per launch.
struct AdamSeg {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  float lr;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float w1,
                                          float b2, float w2, float bc2s, float eps, float step) {
  m = m + w1 * (g - m);
  v = v * b2 + w2 * (g * g);
  const float denom = sqrtf(v) / bc2s + eps;
  p = p - step * (m / denom);
}

__global__ void __launch_bounds__(256)
k_adam(AdamSeg s0, AdamSeg s1, int nblk0, const int32_t* __restrict__ step_count, int step_offset,
       float b1, float b2, float eps) {
  const bool first = (int)blockIdx.x < nblk0;
  const AdamSeg s = first ? s0 : s1;
  const int blk = first ? blockIdx.x : blockIdx.x - nblk0;
  const int nblk = first ? nblk0 : gridDim.x - nblk0;
  const double t = (double)(*step_count + step_offset);
  const float bc1 = (float)(1.0 - pow((double)b1, t));
  const float bc2s = (float)sqrt(1.0 - pow((double)b2, t));
  const float stepsz = (float)((double)s.lr / (double)bc1);
  const float w1 = 1.f - b1, w2 = 1.f - b2;
  const int64_t n4 = s.n / 4;
  for (int64_t i = (int64_t)blk * 256 + threadIdx.x; i < n4; i += (int64_t)nblk * 256) {
    const f32x4 p4 = reinterpret_cast<f32x4*>(s.p)[i];
    const f32x4 g4 = reinterpret_cast<const f32x4*>(s.g)[i];
    const f32x4 m4 = reinterpret_cast<f32x4*>(s.m)[i];
    const f32x4 v4 = reinterpret_cast<f32x4*>(s.v)[i];
    float p[4] = {p4.x, p4.y, p4.z, p4.w}, g[4] = {g4.x, g4.y, g4.z, g4.w};
    float m[4] = {m4.x, m4.y, m4.z, m4.w}, v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) adam_elem(p[e], g[e], m[e], v[e], w1, b2, w2, bc2s, eps, stepsz);
    reinterpret_cast<f32x4*>(s.p)[i] = f32x4{p[0], p[1], p[2], p[3]};
    reinterpret_cast<f32x4*>(s.m)[i] = f32x4{m[0], m[1], m[2], m[3]};
    reinterpret_cast<f32x4*>(s.v)[i] = f32x4{v[0], v[1], v[2], v[3]};
  }
  if (blk == 0 && threadIdx.x < (s.n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    adam_elem(s.p[i], s.g[i], s.m[i], s.v[i], w1, b2, w2, bc2s, eps, stepsz);
  }
}

__global__ void k_inc(int32_t* c) { *c += 1; }

int launch_cls_loss(const float* logits, const int64_t* labels, int B, int K, float lambda_cls,
                    float* dinput, float* dlogits, float* losses, hipStream_t s) {
  PC_REQUIRE(B > 0 && B <= 1024 && K > 0 && K <= 64, "cls_loss: bad shape B=%d K=%d", B, K);
  hipLaunchKernelGGL(k_cls_loss, dim3(1), dim3(1024), 0, s, logits, labels, B, K, lambda_cls,
                     dinput, dlogits, losses);
  PC_HIP_CHECK_LAUNCH("k_cls_loss");
  return PCADV_OK;
}

int launch_disc_loss(const float* dout, int B, const float* soft_gt, const float* soft_nogt,
                     const int32_t* step, uint64_t seed, float lambda_adv, float* ddout,
                     float* losses, hipStream_t s) {
  PC_REQUIRE(B > 0 && B <= 256, "disc_loss: B=%d out of range", B);
  hipLaunchKernelGGL(k_disc_loss, dim3(1), dim3(256), 0, s, dout, B, soft_gt, soft_nogt, step,
                     seed, lambda_adv, ddout, losses);
  PC_HIP_CHECK_LAUNCH("k_disc_loss");
  return PCADV_OK;
}

int launch_lsm_bwd(const float* dinput, const float* ddinput, int B, int K, float* dlogits,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_lsm_bwd, dim3(1), dim3(1024), 0, s, dinput, ddinput, B, K, dlogits);
  PC_HIP_CHECK_LAUNCH("k_lsm_bwd");
  return PCADV_OK;
}

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

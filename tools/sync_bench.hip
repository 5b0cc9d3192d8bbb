// Price of a dependent launch boundary vs an in-launch grid barrier at the
// tail chain's grid sizes (8-128 workgroups).  Standalone diagnostic, not part
// of the library:
//   hipcc -O3 --offload-arch=gfx950 -o build/sync_bench tools/sync_bench.hip
//   build/sync_bench
// (a) a hipGraph of K dependent launches of a G-workgroup kernel whose blocks
//     each read one 4 KB tile the previous launch wrote (the data dependence of
//     the tail chain), time per launch;
// (b) ONE launch of G workgroups running K phases of the same work, separated
//     by a counter barrier (one lane arrives with an agent-scope release
//     add, one lane polls relaxed with s_sleep, then an agent-scope acquire),
//     time per phase.  Every spin is bounded: a timeout sets a flag and the
//     block leaves (the result is then reported invalid, nothing hangs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int TILE = 1024;  // floats per block per phase (4 KB)

// one phase's work: read the tile the previous phase wrote at (blk + 1) % G
// (another workgroup's), add, write this block's tile
__device__ __forceinline__ void phase_body(const float* src, float* dst, int G, int blk) {
  const int from = (blk + 1) % G;
  for (int i = threadIdx.x; i < TILE; i += blockDim.x)
    dst[blk * TILE + i] = src[from * TILE + i] + 1.0f;
}

__global__ void k_step(const float* src, float* dst, int G) { phase_body(src, dst, G, blockIdx.x); }

__global__ void k_persist(float* buf0, float* buf1, int G, int K, unsigned* ctr, unsigned* tmo) {
  __shared__ int fail;
  if (threadIdx.x == 0) fail = 0;
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    const float* src = (k & 1) ? buf1 : buf0;
    float* dst = (k & 1) ? buf0 : buf1;
    phase_body(src, dst, G, blockIdx.x);
    __builtin_amdgcn_s_waitcnt(0);  // this wave's stores issued and done
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(k + 1) * (unsigned)G;
      unsigned spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {
          __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          fail = 1;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __builtin_amdgcn_s_waitcnt(0);  // the invalidate done before the barrier releases
    }
    __syncthreads();
    if (fail) return;
  }
}

int main() {
  const int Ks = 64;
  float *b0, *b1;
  unsigned *ctr, *tmo;
  CK(hipMalloc(&b0, 256 * TILE * 4));
  CK(hipMalloc(&b1, 256 * TILE * 4));
  CK(hipMalloc(&ctr, 256));
  CK(hipMalloc(&tmo, 256));
  CK(hipMemset(b0, 0, 256 * TILE * 4));
  CK(hipMemset(tmo, 0, 256));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int Gs[] = {8, 16, 32, 64, 128};
  const int threads[] = {256, 1024};
  for (int T : threads)
    for (int G : Gs) {
      // (a) graph of K dependent launches
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int k = 0; k < Ks; ++k)
        hipLaunchKernelGGL(k_step, dim3(G), dim3(T), 0, s, (k & 1) ? b1 : b0, (k & 1) ? b0 : b1, G);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      float best_a = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best_a) best_a = ms;
      }
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      // (b) one persistent launch, K phases with a counter barrier
      float best_b = 1e30f;
      for (int r = 0; r < 8; ++r) {
        CK(hipMemsetAsync(ctr, 0, 256, s));
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(k_persist, dim3(G), dim3(T), 0, s, b0, b1, G, Ks, ctr, tmo);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3 && ms < best_b) best_b = ms;
      }
      unsigned t_host = 0;
      CK(hipMemcpy(&t_host, tmo, 4, hipMemcpyDeviceToHost));
      printf("G=%3d T=%4d  launch chain %.2f us/launch   persistent %.2f us/phase%s\n", G, T,
             best_a * 1e3f / Ks, best_b * 1e3f / Ks, t_host ? "  (TIMEOUT: invalid)" : "");
      if (t_host) return 2;
    }
  return 0;
}

// Probe: does a CU-masked stream let a one-workgroup kernel (16 waves, ~147 KB LDS, like k_build_small) start while
// a persistent kernel fills every other CU?  Hog: a grid that fills the CUs of its stream's mask and spins for
// ~4 ms.  1 ms after the hog starts, the small kernel is launched on a second stream; it records when it began.
// Modes: unmasked (both streams on every CU) / masked (hog: all CUs but CU 0; small: CU 0 only).
//   hipcc --offload-arch=gfx950 -O2 scripts/cumask_probe.hip -o scripts/cumask_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void __launch_bounds__(256) hog(unsigned long long* t0, unsigned long long spin) {
  const unsigned long long s = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) t0[0] = s;
  while (__builtin_amdgcn_s_memrealtime() - s < spin) __builtin_amdgcn_s_sleep(10);
}

__global__ void __launch_bounds__(1024) small(unsigned long long* t) {
  __shared__ float lds[36 * 1024];
  const unsigned long long s = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) { t[1] = s; t[2] = (unsigned long long)lds[5]; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  printf("CUs %d\n", ncu);
  unsigned long long* t;
  CK(hipMalloc(&t, 64));
  for (int masked = 0; masked < 2; masked++) {
    hipStream_t a, b;
    std::vector<uint32_t> ma((ncu + 31) / 32, 0xFFFFFFFFu), mb((ncu + 31) / 32, 0u);
    if (masked) { ma[0] &= ~1u; mb[0] = 1u; }
    CK(hipExtStreamCreateWithCUMask(&a, (uint32_t)ma.size(), ma.data()));
    CK(hipExtStreamCreateWithCUMask(&b, (uint32_t)mb.size(), mb.data()));
    for (int rep = 0; rep < 2; rep++) {
      CK(hipMemset(t, 0, 64));
      CK(hipDeviceSynchronize());
      const int blocks = (ncu - masked) * 8;  // 8 x 4 waves per CU: every wave slot of the hog's CUs
      hipLaunchKernelGGL(hog, dim3(blocks), dim3(256), 0, a, t, 400000ull);  // 4 ms at 100 MHz
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
      hipLaunchKernelGGL(small, dim3(1), dim3(1024), 0, b, t);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned long long h[3];
      CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
      printf("%s rep %d: small kernel began %.3f ms after the hog (hog spins 4.000 ms)\n", masked ? "masked" : "unmasked",
             rep, (double)(long long)(h[1] - h[0]) / 1e5);
    }
    CK(hipStreamDestroy(a));
    CK(hipStreamDestroy(b));
  }
  return 0;
}

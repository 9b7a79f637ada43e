// rcp_exhaustive.hip -- is v_rcp_f32 + one FMA Newton step the correctly rounded 1/x on gfx950?
//
// The triangle test (prt_traverse.h mt_test) and safercp divide 1 by a float; the oracle does the same in C,
// so the GPU must return the IEEE correctly rounded quotient.  hipcc's division is a ~12-instruction
// div_scale / rcp / fma / div_fmas / div_fixup sequence.  This program compares, for every float bit pattern
// x, r1 = fma(fma(-x, r0, 1), r0, r0) with r0 = v_rcp_f32(x) against 1.0f / x, and reports the mismatches
// by magnitude class.  Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -o rcp_exhaustive
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void k_check(uint32_t lo_exp_bits, unsigned long long* counts, uint32_t* first) {
  // counts[0]: mismatches with |x| in [2^-125, 2^125] (results normal), counts[1]: elsewhere (finite x)
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long c0 = 0, c1 = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
    const uint32_t b = (uint32_t)i;
    const float x = __uint_as_float(b);
    if (!isfinite(x) || x == 0.0f) continue;
    const float r0 = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r0, 1.0f);
    const float r1 = __builtin_fmaf(e, r0, r0);
    const float ref = 1.0f / x;
    if (__float_as_uint(r1) != __float_as_uint(ref)) {
      const uint32_t ex = (b >> 23) & 0xFFu;
      if (ex >= lo_exp_bits && ex <= 254u - lo_exp_bits) {
        c0++;
        atomicCAS(first, 0u, b);
      } else {
        c1++;
      }
    }
  }
  if (c0) atomicAdd(&counts[0], c0);
  if (c1) atomicAdd(&counts[1], c1);
}

int main() {
  unsigned long long* d;
  uint32_t* f;
  if (hipMalloc(&d, 2 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&f, 4) != hipSuccess) return 2;
  (void)hipMemset(d, 0, 2 * sizeof(unsigned long long));
  (void)hipMemset(f, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(256 * 8 * 4), dim3(256), 0, 0, 2u, d, f);  // exponent field in [2, 252]
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  unsigned long long h[2];
  uint32_t first;
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&first, f, 4, hipMemcpyDeviceToHost);
  std::printf("rcp+newton vs 1/x: %llu mismatches for |x| in [2^-125, 2^126) (first 0x%08x), %llu outside\n", h[0],
              first, h[1]);
  return h[0] == 0 ? 0 : 1;
}

// fetch_calibration.hip -- calibrates rocprofv3's FETCH_SIZE against known byte counts on gfx950 for the access
// shapes of the traversal kernel (MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of the bytes of a wide coalesced
// streaming read; is the same true of random gathers?).  Each kernel reads every byte of its input exactly once,
// from a buffer larger than the 256 MiB Infinity Cache, with a 768 MiB write to another buffer in between (so no
// input line is cache-resident when its kernel starts):
//
//   k_stream    coalesced float4 stream over 1 GiB                                   (the guide's reference shape)
//   k_lines128  one random 128-B line per lane (8 x 16-B loads), a permutation of 1 GiB
//   k_rec80     one random 80-B record per lane (5 x 16-B loads; the Node8 size, packed at 80-B stride), 640 MiB
//   k_gather16  one random 16-B item per lane, a permutation of 1 GiB (several items share a line: over-fetch
//               is physical here, not a counter artefact)
//
// Each lane writes one float (4 B) so the loads are live.  The program prints the known bytes per kernel as JSON;
// scripts/summarize_fetch_calibration.py divides them by the FETCH_SIZE / WRITE_SIZE of the --pmc passes.
// build: hipcc -O3 --offload-arch=gfx950 scripts/fetch_calibration.hip -o scripts/bin/fetch_calibration
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

// a bijection of [0, 2^k): odd multiplier + offset modulo a power of two
__device__ __forceinline__ uint32_t perm(uint32_t i, uint32_t mask) { return (i * 2654435761u + 0x9E3779B9u) & mask; }

__global__ void k_stream(const float4* __restrict__ in, float* __restrict__ out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 v = in[i];
  out[i] = v.x + v.y + v.z + v.w;
}

__global__ void k_lines128(const float4* __restrict__ in, float* __restrict__ out, uint32_t n, uint32_t mask) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4* p = in + 8ull * perm(i, mask);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; k++) { const float4 v = p[k]; s += v.x + v.y + v.z + v.w; }
  out[i] = s;
}

__global__ void k_rec80(const float4* __restrict__ in, float* __restrict__ out, uint32_t n, uint32_t mask) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4* p = in + 5ull * perm(i, mask);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 5; k++) { const float4 v = p[k]; s += v.x + v.y + v.z + v.w; }
  out[i] = s;
}

__global__ void k_gather16(const float4* __restrict__ in, float* __restrict__ out, uint32_t n, uint32_t mask) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 v = in[perm(i, mask)];
  out[i] = v.x + v.y + v.z + v.w;
}

int main() {
  const size_t GiB = 1ull << 30;
  float4* in = nullptr;
  float* out = nullptr;
  void* flush = nullptr;
  CK(hipMalloc(&in, GiB));
  CK(hipMalloc(&out, (1ull << 26) * sizeof(float)));
  CK(hipMalloc(&flush, 768ull << 20));
  CK(hipMemset(in, 0x3c, GiB));
  auto flush_caches = [&]() {
    CK(hipMemset(flush, 1, 768ull << 20));
    CK(hipDeviceSynchronize());
  };
  const uint32_t B = 256;
  const uint32_t n_stream = 1u << 26, n_lines = 1u << 23, n_rec = 1u << 23, n_g16 = 1u << 26;
  for (int rep = 0; rep < 2; rep++) {
    flush_caches();
    k_stream<<<n_stream / B, B>>>(in, out, n_stream);
    flush_caches();
    k_lines128<<<n_lines / B, B>>>(in, out, n_lines, n_lines - 1);
    flush_caches();
    k_rec80<<<n_rec / B, B>>>(in, out, n_rec, n_rec - 1);
    flush_caches();
    k_gather16<<<n_g16 / B, B>>>(in, out, n_g16, n_g16 - 1);
    CK(hipDeviceSynchronize());
  }
  std::printf("{\"k_stream\": {\"read\": %zu, \"write\": %zu}, \"k_lines128\": {\"read\": %zu, \"write\": %zu}, "
              "\"k_rec80\": {\"read\": %zu, \"write\": %zu}, \"k_gather16\": {\"read\": %zu, \"write\": %zu}}\n",
              (size_t)n_stream * 16, (size_t)n_stream * 4, (size_t)n_lines * 128, (size_t)n_lines * 4,
              (size_t)n_rec * 80, (size_t)n_rec * 4, (size_t)n_g16 * 16, (size_t)n_g16 * 4);
  CK(hipFree(in));
  CK(hipFree(out));
  CK(hipFree(flush));
  return 0;
}

// isa_counts.hip -- ISA instruction counts of one Node8 visit (node8_hits) and one triangle test (mt_test), each
// compiled alone into a kernel with the product's flags (csrc/Makefile).  scripts/isa_counts.py compiles this to
// gfx950 assembly and counts the VALU / SALU / memory instructions of each kernel body -> profiles/isa_counts.json.
#include "../physically-based-ray-tracer_amd/csrc/prt_traverse8.h"

using namespace prt;

__global__ void k_isa_node8(const Node8* __restrict__ nodes, const float* __restrict__ ray, uint32_t* out) {
  const uint32_t i = threadIdx.x;
  const uint4* np = reinterpret_cast<const uint4*>(nodes + i);
  const V3 O = v3(ray[0], ray[1], ray[2]), rD = v3(ray[3], ray[4], ray[5]);
  out[i] = node8_hits(np[0], np[2], np[3], np[4], O, rD, ray[6]);
}

__global__ void k_isa_tri(const TriMT* __restrict__ tris, const float* __restrict__ ray, float* out) {
  const uint32_t i = threadIdx.x;
  const V3 O = v3(ray[0], ray[1], ray[2]), D = v3(ray[3], ray[4], ray[5]);
  float t, u, v;
  uint32_t prim;
  const bool h = mt_test(tris + i, O, D, t, u, v, prim);
  out[i] = h ? t + u + v : 0.0f;
}

// rt_bvh.hpp -- device-side BVH build (rt_bvh.hip), called by rtBuildBVH (rt_capi.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/rt_cl_types.h"

namespace rtb {

// device scratch needed to build over n triangles
size_t scratch_bytes(uint32_t n);

// Builds over tris[0, n) (file order) on `st`: permutes tris into leaf order in place and
// writes *n_nodes (<= 2n - 1) CLLinearBVHNode records to `nodes` (synchronises once to read
// the node count; PLOC once per clustering round).  max_prims >= 1.  method: 0 linear BVH
// (Karras radix tree), 1 PLOC.
hipError_t build(rt_cl_triangle* tris, uint32_t n, uint32_t max_prims, rt_cl_bvh_node* nodes, uint32_t* n_nodes,
                 void* scratch, hipStream_t st, int method);

}  // namespace rtb

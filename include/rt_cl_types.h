/*
 * rt_cl_types.h -- byte layout of the buffers the hot path consumes.
 *
 * Layout contract of /root/reference/CLshared_structs.hpp:7-87 as seen by the device:
 * every OpenCL float3 occupies a 16-byte slot (x, y, z, pad).  A host written against
 * the reference (CLTriangle/CLVertex/CLLinearBVHNode/CLMaterial built from its own
 * float3 class, CLmathlib.hpp:18-54, which is 16 bytes) produces exactly these bytes.
 * Plain C so it can be shared by C, C++ and HIP translation units.
 */
#ifndef RT_CL_TYPES_H
#define RT_CL_TYPES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_float3 { float x, y, z, w; } rt_float3;            /* OpenCL float3 */

typedef struct rt_cl_vertex {                                          /* CLVertex, 80 B */
    rt_float3 position, uv, normal, tangent_s, tangent_t;
} rt_cl_vertex;

typedef struct rt_cl_triangle {                                        /* CLTriangle, 256 B */
    rt_cl_vertex v1, v2, v3;
    uint32_t mtlIndex;
    uint32_t padding[3];
} rt_cl_triangle;

typedef struct rt_cl_bounds { rt_float3 pmin, pmax; } rt_cl_bounds;    /* CLBounds3, 32 B */

typedef struct rt_cl_bvh_node {                                        /* CLLinearBVHNode, 48 B */
    rt_cl_bounds bounds;
    uint32_t offset;      /* leaf: first primitive; interior: second child */
    uint16_t nPrimitives; /* 0 -> interior */
    uint8_t axis;         /* interior: split axis */
    uint8_t pad[9];
} rt_cl_bvh_node;

typedef struct rt_cl_material {                                        /* CLMaterial, 64 B */
    rt_float3 diffuse, specular, emission;
    uint32_t type;
    float roughness;
    float ior;
    int32_t padding;
} rt_cl_material;

#ifdef __cplusplus
static_assert(sizeof(rt_float3) == 16, "float3 slot");
static_assert(sizeof(rt_cl_vertex) == 80, "CLVertex");
static_assert(sizeof(rt_cl_triangle) == 256, "CLTriangle");
static_assert(sizeof(rt_cl_bvh_node) == 48, "CLLinearBVHNode");
static_assert(sizeof(rt_cl_material) == 64, "CLMaterial");
static_assert(offsetof(rt_cl_triangle, mtlIndex) == 240, "CLTriangle.mtlIndex");
static_assert(offsetof(rt_cl_bvh_node, offset) == 32, "node.offset");
static_assert(offsetof(rt_cl_bvh_node, nPrimitives) == 36, "node.nPrimitives");
static_assert(offsetof(rt_cl_bvh_node, axis) == 38, "node.axis");
}
#else
_Static_assert(sizeof(rt_cl_triangle) == 256, "CLTriangle");
_Static_assert(sizeof(rt_cl_bvh_node) == 48, "CLLinearBVHNode");
_Static_assert(sizeof(rt_cl_material) == 64, "CLMaterial");
#endif

#endif /* RT_CL_TYPES_H */

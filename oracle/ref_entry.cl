/*
 * ref_entry.cl -- test harness around the UNMODIFIED reference kernel (test infrastructure).
 *
 * Built by `make -C oracle ref` with the image's OpenCL compiler for gfx950: the
 * reference source /root/reference/kernel_bvh.cl is #included in place (nothing is
 * copied or edited), so the code object oracle/_ref/kernel_bvh_*.co contains the
 * reference's own KernelEntry (kernel_bvh.cl:415-456).  One extra entry point is added
 * here: PrimaryHitEntry runs the reference's own CreateRay (:386-403) and Intersect
 * (:171-219) for one frame's primary rays and stores the hit primitive index
 * (`isect.object - triangles`, -1 = miss) and isect.t -- values the reference computes
 * but never writes out.
 */
#include "kernel_bvh.cl"

__kernel void PrimaryHitEntry(__global int* hitIds, __global float* hitT,
                              __global CLTriangle* triangles, __global CLLinearBVHNode* nodes,
                              __global CLMaterial* materials, unsigned int width,
                              unsigned int height, unsigned int frameCount, float3 cameraPos,
                              float3 cameraFront, float3 cameraUp)
{
    Scene scene = {triangles, nodes, materials, 1u, 0, 1.0f, cameraPos, cameraFront, cameraUp};
    unsigned int seed = get_global_id(0) + HashUInt32(frameCount);
    Ray ray = CreateRay(width, height, cameraPos, cameraFront, cameraUp, &seed);
    IntersectData isect = Intersect(&ray, &scene);
    hitIds[get_global_id(0)] = isect.hit ? (int)(isect.object - triangles) : -1;
    hitT[get_global_id(0)] = isect.t;
}

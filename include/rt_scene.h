/*
 * rt_scene.h -- C ABI of the host scene pipeline (librt_scene.so).
 *
 * Restates the reference host path that produces the three device arrays:
 *   CLOBJloader::Load / LoadTriangles / LoadMaterials   (CLOBJloader.cpp:10-176)
 *   CLBVHScene::CreateBVHTrees / RecursiveBuild / FlattenBVHTree (CLBVHnode.cpp:7-207)
 * The arrays come out in the rt_cl_types.h layout (CLTriangle 256 B in BVH leaf order,
 * CLLinearBVHNode 48 B in depth-first order, CLMaterial 64 B), ready for
 * rtCreateBuffer(... RT_MEM_COPY_HOST_PTR ...) exactly as CLBVHScene::SetupBuffers
 * (CLBVHnode.cpp:209-236) hands them to clCreateBuffer.
 *
 * All functions return 0 on success or a negative CL-style status (rt_status.h).
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <stddef.h>
#include <stdint.h>

#include "rt_cl_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_scene rt_scene;

/* CLOBJloader::Load(filename, maxPrimitivesInNode) followed by
 * CLBVHScene::CreateBVHTrees(maxPrimitivesInNode) (CLEngineBase.cpp:173-179).
 * The .mtl file is the .obj path with its last four characters replaced by ".mtl"
 * (CLOBJloader.cpp:18-21). */
int rtsLoadOBJ(const char* obj_path, unsigned max_prims_in_node, rt_scene** out);

/* Load only (no BVH): triangles in file order, as CLOBJloader leaves m_Triangles. */
int rtsLoadOBJUnbuilt(const char* obj_path, rt_scene** out);

/* Build a scene from caller triangles (file order) + materials, then CreateBVHTrees. */
int rtsBuildFromTriangles(const rt_cl_triangle* tris, size_t n_tris,
                          const rt_cl_material* mats, size_t n_mats,
                          unsigned max_prims_in_node, rt_scene** out);

/* Borrowed views of the arrays (valid until rtsRelease). */
int rtsGetTriangles(const rt_scene* s, const rt_cl_triangle** tris, size_t* count);
int rtsGetNodes(const rt_scene* s, const rt_cl_bvh_node** nodes, size_t* count);
int rtsGetMaterials(const rt_scene* s, const rt_cl_material** mats, size_t* count);

/* Tree statistics: maximum leaf depth (root = 0), leaf count, max primitives per leaf. */
int rtsGetTreeStats(const rt_scene* s, unsigned* max_depth, unsigned* n_leaves,
                    unsigned* max_leaf_prims);

/* Wrap caller arrays that are already built (BVH order + flattened nodes), e.g. to cache a
 * scene built elsewhere.  Node child / leaf ranges are validated. */
int rtsFromArrays(const rt_cl_triangle* tris, size_t n_tris, const rt_cl_bvh_node* nodes, size_t n_nodes,
                  const rt_cl_material* mats, size_t n_mats, unsigned max_prims_in_node, rt_scene** out);

/* Binary scene cache: the three device arrays exactly as built, so a large
 * OBJ is parsed and its BVH built once.  Format: "RTSCENE1", u32 version, u32
 * maxPrimitivesInNode, u64 triangle / node / material counts, the raw arrays, u64 FNV-1a of
 * everything before it.  A bad magic, size or checksum is RT_PARSE_ERROR. */
int rtsSaveScene(const rt_scene* s, const char* path);
int rtsLoadScene(const char* path, rt_scene** out);

void rtsRelease(rt_scene* s);

#ifdef __cplusplus
}
#endif

#endif /* RT_SCENE_H */

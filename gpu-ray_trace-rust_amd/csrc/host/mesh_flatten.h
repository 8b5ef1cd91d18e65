// mesh_flatten.h — host precompute of mesh triangles for the device (not part of the C ABI).
#pragma once

#include <cstdint>
#include <vector>

#include "../../../include/rt_abi.h"

namespace rth {

struct FlatPrim {
    float base_factor[3];
    int32_t base_tex;    // -1: factor only (RgbFromMesh, mesh/triangle.rs:166-178)
    int32_t normal_tex;  // -1: interpolated vertex normals (mesh/triangle.rs:148-155)
    int32_t mr_tex;      // -1: metal/rough factors (mesh/triangle.rs:193-200)
    float metal, rough;
};

struct FlatTri {
    uint32_t prim;
    uint32_t v[3];       // global vertex indices (pools below)
    float m[9];          // row-major normal transform (x normal_scale with a normal map)
    uint32_t _pad[3];
};
static_assert(sizeof(FlatTri) == 64, "FlatTri is one 64-byte record");

struct MeshFlat {
    std::vector<FlatPrim> prims;
    std::vector<FlatTri> tris;      // renderable order: mesh, primitive, triangle
    std::vector<float> verts;       // 3 x float4 per triangle (pre-gathered positions)
    std::vector<float> norms;       // float4 per global vertex
    std::vector<float> base_uv, normal_uv, mr_uv;  // float2 per global vertex (0 when absent)
};

int flatten_meshes(const rt_scene_desc* sc, MeshFlat* out);

}  // namespace rth

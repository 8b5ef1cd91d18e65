// host_internal.h — shared declarations of the host side of the boundary (not part of the ABI).
#pragma once

#include <cstdint>
#include <vector>

#include "../../../include/rt_abi.h"

namespace rth {

// Renderable kinds on the device.  Non-mesh kinds equal RT_ELEM_*; mesh triangles follow.
enum : uint32_t { RT_KIND_SPHERE = 0, RT_KIND_FREE_TRI = 1, RT_KIND_CUBE_MAP = 2, RT_KIND_MESH_TRI = 3 };

// One renderable in reference order (draw_scene.rs:57-58): kind, index into its kind's array
// (mesh triangles: running index over meshes/prims/triangles), its Aabb if it has one.
struct Renderable {
    uint32_t kind;
    uint32_t index;
    bool has_aabb;
    float lo[3], hi[3];
};

int gather_renderables(const rt_scene_desc* sc, std::vector<Renderable>* out);

}  // namespace rth

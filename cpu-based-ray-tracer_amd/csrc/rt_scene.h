// rt_scene.h -- host-side scene path: OBJ input, reference-identical two-level BVH build, and the
// flattening into the HBM layout of rt_layout.h.  C++20, no HIP dependency.
#ifndef RT_SCENE_H
#define RT_SCENE_H
#include <cstdint>
#include <string>
#include <vector>

#include "rt_layout.h"

namespace rt {

struct F3 { float x, y, z; };

struct MaterialDesc { F3 albedo; F3 emission; };

struct MeshDesc {
    std::vector<float> raw;   // de-indexed objl positions, 9 floats per triangle, BEFORE the 0.01 scale
    MaterialDesc material;
    std::string name;
};

// Flattened, upload-ready scene (rt_layout.h).
struct FlatScene {
    rt_scene_header hdr{};
    std::vector<float> nodes, tris, mats, lnodes, ltris;   // float4-granular
    // per-node debug view (tests): box, area, left, right, tri, mesh, top-level flag
    std::vector<float> dbg_node_f;    // 7 per node
    std::vector<int32_t> dbg_node_i;  // 5 per node
    std::vector<float> dbg_tri_f;     // 13 per tri (a b c n area)
    std::vector<int32_t> dbg_tri_i;   // 2 per tri (mesh, material)
};

class SceneBuilder {
public:
    // objl::Loader::LoadFile subset (MC/OBJ_Loader.h:434-720): positions of the first mesh, de-indexed.
    static bool load_obj_positions(const std::string& path, std::vector<float>& raw, std::string& err);
    // The Cornell box exactly as Renderer::Renderer() builds it (MC/Renderer.cpp:26-57), from the
    // box's public measurement data (MC/cornellbox/*.obj carry the same numbers).
    void add_cornell_box();
    static std::vector<MeshDesc> cornell_box_meshes();
    int add_mesh(MeshDesc m);
    // Renderer::GenerateBVH (MC/Renderer.h:83-86) + TriangleMesh's per-mesh BVH (MC/TriangleMesh.h:185)
    bool build(FlatScene& out, std::string& err) const;
    size_t num_meshes() const { return meshes_.size(); }
    const std::vector<MeshDesc>& meshes() const { return meshes_; }

private:
    std::vector<MeshDesc> meshes_;
};

}  // namespace rt
#endif

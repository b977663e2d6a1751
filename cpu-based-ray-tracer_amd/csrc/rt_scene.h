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

// albedo: MC diffuse_coefficient (path tracing) / BV diffuse color (Whitted); phong_diffuse: BV only
struct MaterialDesc { F3 albedo; F3 emission; float phong_diffuse = 0.0f; };

struct MeshDesc {
    std::vector<float> raw;   // de-indexed objl positions, 9 floats per triangle, BEFORE the scale
    MaterialDesc material;
    std::string name;
    // vertex = scale * p (MC/TriangleMesh.h:165-168, scale 0.01), or with an offset
    // vertex = offset + scale * p (BV/TriangleMesh.h:124-127)
    float scale = 0.01f;
    bool has_offset = false;
    F3 offset{0.0f, 0.0f, 0.0f};
    // a sphere entity of the path-traced scene instead of a mesh (Whitted::Sphere, MC/Sphere.h:16-108): raw is empty
    bool sphere = false;
    F3 center{0.0f, 0.0f, 0.0f};
    float radius = 0.0f;
};

struct PointLight { F3 position; F3 radiance; };

// An entity of the Whitted Style Ray Tracer's world (WH/Entity.h:16-57, WH/Sphere.h, WH/TriangleMesh.h).
// nature: 0 Reflective, 1 Reflective_Refractive, 2 Diffuse_Glossy (WH/WhittedUtilities.h:18-23).
struct WorldEntity {
    int kind = 0;                       // 0 sphere, 1 indexed triangle mesh
    F3 center{0, 0, 0};
    float radius = 0.0f;
    std::vector<F3> vertices;           // mesh: vertex positions
    std::vector<uint32_t> indices;      // mesh: 3 per triangle
    std::vector<float> uv;              // mesh: 2 per vertex
    int nature = 2;
    float refractive_index = 1.3f, phong_diffuse = 0.8f, phong_specular = 0.2f, specular_size_factor = 25.0f;
    F3 diffuse_color{0.2f, 0.2f, 0.2f};
};

// Flattened, upload-ready scene (rt_layout.h).
struct FlatScene {
    rt_scene_header hdr{};
    std::vector<float> nodes, tris, mats, lnodes, ltris, wmats, plights;   // float4-granular
    std::vector<float> went, wtris;                                       // Whitted world (C1)
    std::vector<float> lboxes;                                            // distinct leaf boxes (small scenes)
    // split trace (larger scenes, the vertex kernel's BVH variant): the subtree [split_root, split_end) of
    // the DFS pre-order is walked; the <= 32 leaves outside it are tested by their distinct leaf boxes
    // (sboxes: the lboxes layout, the masks over outside slots), slot k = the k-th outside leaf in DFS
    // order = triangle stri[k]; split_root = 0: no split
    std::vector<float> sboxes;
    std::vector<int32_t> stri;
    uint32_t split_root = 0, split_end = 0;
    // split scenes: the walked subtree in 8 near-first pre-orders (one per direction octant), node k of
    // ordering o at [(o * (split_end - split_root) + k) * 8], indices as in `nodes`; the nodes layout with
    // each box as (near.xyz, far.x)(far.y, far.z, skip, tri), near/far the planes a ray of octant o meets
    // first/last (x: (hi, lo) when bit 0 -- d.x < 0 -- is set)
    std::vector<float> wcopies;
    // Whitted scenes (point lights): the whole tree in 8 near-first pre-orders, node k of ordering o at
    // [(o * n_nodes + k) * 8] (empty: the kernel walks `nodes`)
    std::vector<float> worders;
    // the same orderings in 16 bytes per node (round 6): each plane as an IEEE half rounded OUTWARD (a low plane
    // down, a high plane up: the decoded box contains the exact one), (near.x | far.x << 16, near.y | far.y << 16,
    // near.z | far.z << 16, skip | internal, or 0x80000000 | triangle for a leaf, whose successor is the next
    // node); built when every leaf's box is its triangle's vertex box (`tabc` holds the vertices for the exact
    // leaf test); empty otherwise
    std::vector<uint32_t> worders_h;
    std::vector<float> tabc;   // the triangles' vertices by slot, 3 float4 each (built when hdr.has_vboxes)
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
    // Renderer::Add(new Whitted::Sphere(center, radius, material)) (MC/Sphere.h:19-23): an entity like a mesh
    int add_sphere(const F3& center, float radius, const MaterialDesc& m);
    // Renderer::Add(std::unique_ptr<PointLightSource>), BV/Renderer.h:88-97
    void add_point_light(const PointLight& l) { lights_.push_back(l); }
    void set_sky(const F3& c) { sky_ = c; }
    // World::Add(std::unique_ptr<Entity>) (WH/World.h:37-45)
    int add_world_entity(WorldEntity e) { world_.push_back(std::move(e)); return (int)world_.size() - 1; }
    // the world of the Whitted Style Ray Tracer's Renderer::Renderer() (WH/Renderer.cpp:27-49)
    void add_two_spheres_scene();
    // Renderer::GenerateBVH (MC/Renderer.h:83-86) + TriangleMesh's per-mesh BVH (MC/TriangleMesh.h:185)
    bool build(FlatScene& out, std::string& err) const;
    size_t num_meshes() const { return meshes_.size(); }
    const std::vector<MeshDesc>& meshes() const { return meshes_; }

private:
    std::vector<MeshDesc> meshes_;
    std::vector<PointLight> lights_;
    std::vector<WorldEntity> world_;
    F3 sky_{0.2f, 0.7f, 0.8f};   // BV/Renderer.h:189
};

}  // namespace rt
#endif

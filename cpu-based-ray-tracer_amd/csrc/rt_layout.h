// rt_layout.h -- device-side scene layout shared by the host builder (rt_scene.cpp) and the
// HIP kernels (rt_kernels.hip).  Plain C structs, no HIP types.
//
// HBM layout (all arrays 16-byte aligned, float4-granular):
//
//  nodes   : 2 x float4 per BVH node, flattened two-level BVH in DFS pre-order
//            (top-level BVH over meshes, each top-level leaf replaced by the mesh's own BVH root;
//            exact because a mesh's top-level box equals its mesh-root box,
//            MC/TriangleMesh.h:173-178 vs MC/BVH.h:155,208).
//              q0 = (lo.x, lo.y, lo.z, hi.x)
//              q1 = (hi.y, hi.z, bits(skip), bits(tri))
//            skip = index of the next node in DFS pre-order after this node's subtree (== count at
//            the end); tri = triangle slot for leaves, -1 for internal nodes.  An internal node's
//            left child is the next node (i+1).  A miss or a finished leaf continues at `skip`,
//            so a stackless walk visits exactly the nodes the reference's recursion visits
//            (BVH::traverse_BVH_from_node, MC/BVH.h:82-101).
//  tris    : 4 x float4 per triangle, in DFS leaf order (slot == flattened leaf index)
//              q0 = (a.xyz, bits(material)), q1 = (e1 = b-a, bits(primitive id)), q2 = (e2 = c-a, 0), q3 = (n.xyz, 0)
//            (primitive id: 1 + creation index over all meshes, the Denoiser's G-buffer id, DN/TriangleMesh.h:54-62)
//            (Moller-Trumbore reads q0..q2 = 48 B; shading reads q3)
//            a sphere slot (Whitted::Sphere, MC/Sphere.h:16-108; round 6): q0 = (center.xyz, bits(material)),
//            q1 = (radius^2, radius, 0, bits(primitive id)), q2 = (0, 0, 0, bits(1): the sphere flag), q3 = 0
//            (the normal is normalize(location - center) at the hit)
//  mats    : 2 x float4 per material: (brdf = albedo/PI, emitting), (emission, 0)
//  lnodes  : light-mesh BVH for area sampling (BVH::Sampling_from_node, MC/BVH.h:114-129):
//            1 x float4 per node (area, bits(left), bits(right), bits(light_tri)), root = 0
//  ltris   : 4 x float4 per light triangle: (a, skip), (b, 0), (c, 0), (n, area); skip: bits of the
//            scene triangles (<= 32) a shadow ray toward this triangle cannot be blocked by (rt_scene.cpp)
//  wmats   : Whitted-style shading (BVH Ray Tracer, BV/Renderer.cpp:172-229): 1 x float4 per
//            material: (diffuse color, phong_diffuse)
//  plights : point lights in insertion order (BV/LightSource.h, BV/Renderer.cpp:38-39):
//            2 x float4 per light: (position, 0), (radiance, 0)
//  went    : the Whitted Style Ray Tracer's world (config C1, WH/World.h): entities in insertion
//            order, intersected brute force (WH/Renderer.h:109-140), 4 x float4 per entity:
//              q0 = (bits(kind: 0 sphere, 1 triangle mesh), bits(material nature), bits(first wtri), bits(n tris))
//              q1 = (sphere center.xyz, radius)
//              q2 = (radius^2, refractive_index, phong_diffuse, phong_specular)
//              q3 = (diffuse_color.xyz, specular_size_factor)          (WH/Entity.h:49-55)
//  wtris   : triangles of the world's meshes, 4 x float4 per triangle:
//              (v1.xyz, uv1.x), (v2.xyz, uv1.y), (v3.xyz, uv2.x), (uv2.y, uv3.x, uv3.y, 0)
#ifndef RT_LAYOUT_H
#define RT_LAYOUT_H
#include <stdint.h>

#define RT_NODE_QUADS 2
#define RT_TRI_QUADS 4
#define RT_MAT_QUADS 2
#define RT_LTRI_QUADS 4

typedef struct {
    uint32_t n_nodes, n_tris, n_mats, n_lnodes, n_ltris;
    int32_t light_mesh;        // first emissive mesh in insertion order (MC/Renderer.h:169-179), -1 if none
    float light_area;          // light mesh BVH root mesh_area (pdf = 1/area, MC/BVH.h:106)
    float light_emission[3];   // emission of the light mesh material (MC/TriangleMesh.h:195)
    uint32_t max_depth;        // deepest node level (for diagnostics)
    uint32_t n_plights;        // point lights (Whitted shading)
    float sky[3];              // Whitted miss color (BV/Renderer.h:189)
    uint32_t n_went, n_wtris;  // Whitted world (config C1): entities and mesh triangles
    int32_t max_bounce_depth;  // WH/World.h:55
    float intersection_correction;   // WH/World.h:56
    uint32_t n_lboxes;         // distinct leaf boxes of a small scene (<= 64 triangles), 0 otherwise
    uint32_t has_vboxes;       // every leaf box is its triangle's vertex box (FlatScene::tabc holds the vertices)
    uint32_t n_spheres;        // sphere entities (their slots in `tris` carry the sphere flag)
} rt_scene_header;

// tabc (when hdr.has_vboxes; the Whitted half-plane walk's exact leaf boxes): 3 x float4 per triangle slot:
//   (a, bits(material)), (b, bits(primitive id)), (c, 0); Moller-Trumbore takes e1 = b - a, e2 = c - a (the same
//   correctly rounded floats as `tris`).  (Round 6: the 16-bit compact BVH "qnodes" and its normals are gone.)

// lboxes (small scenes: the vertex kernel's leaf-box trace, the megakernel's coherent trace): 2 float4
// per distinct leaf box, (lo.x, hi.x, lo.y, hi.y)(lo.z, hi.z, bits of the mask of its triangles 0-31,
// bits of the mask of triangles 32-63) -- each axis' planes adjacent, so a scalar load yields the
// (lo, hi) pair of a packed subtraction
#define RT_LBOX_QUADS 2

#define RT_WENT_QUADS 4
#define RT_WTRI_QUADS 4
#define RT_WORLD_SPHERE 0
#define RT_WORLD_MESH 1

#endif

// scene.h -- C++ host mirror of the reference's RayTracing::Scene / Camera / BVH
// (RayTracing/Scene.{h,cpp}, RayTracing/BVH.{h,cpp}).  Same method names and semantics,
// so a host written against the reference drives this path unchanged; device memory goes
// through the C-ABI shim (include/rt_abi.h) instead of CUDA::DeviceMemory.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_host_math.h"

namespace RayTracing {

using rtm::f3;
using rth::mat4;

// Scene.h:21-26
enum class DirtyFlagValue : uint32_t { Samples = 1 << 0, SceneMemory = 1 << 1, BVH = 1 << 2 };
typedef uint32_t DirtyFlags;

// RAII device buffer with the reference's DeviceMemory contract (utils/CUDAHelper.h:114-156):
// allocation failure throws std::runtime_error("allocation failed").
class DeviceMemory {
    void* memory = nullptr;
    size_t size = 0;

   public:
    explicit DeviceMemory(size_t size);
    ~DeviceMemory();
    DeviceMemory(const DeviceMemory&) = delete;
    DeviceMemory& operator=(const DeviceMemory&) = delete;
    size_t GetSize() const { return size; }
    void* GetMemory() const { return memory; }
};

// Scene.h:33-71 / Scene.cpp:15-36
struct Camera : public GPUCamera {
    Camera();
    void SetViewportSize(float w, float h) { viewport_w = w, viewport_h = h; }
    void SetPosition(f3 p) { origin[0] = p.x, origin[1] = p.y, origin[2] = p.z; }
    void SetXAndle(float v) { angle_x = v; }
    void SetYAndle(float v) { angle_y = v; }
    float GetXAngle() const { return angle_x; }
    float GetYAngle() const { return angle_y; }
    void Update();

   private:
    float viewport_w = 1, viewport_h = 1;
    float angle_x = 0, angle_y = 0, fov_y = 90;
    mat4 transform, projection, view;
};

// Scene.h:74-85
struct Material : public GPUMaterial {
    Material(f3 albedo, f3 emissive);
    explicit Material(f3 albedo) : Material(albedo, f3{0, 0, 0}) {}
    Material() : Material(f3{0, 0, 0}) {}
};

// BVH.h:17-42 / BVH.cpp
class BVH {
    struct Triangle {
        f3 centroid;
        uint32_t index;
    };
    std::vector<GPUBVHNode> nodes;
    std::vector<Triangle> triangles;
    const GPUVertex* vertices = nullptr;
    const GPUFace* faces = nullptr;
    uint32_t root_node_id = 0;
    uint32_t nodes_used = 1;
    std::vector<uint32_t> face_indices;
    int max_depth = 0;

    void UpdateBounds(uint32_t node);
    void Subdivide(uint32_t node, int depth);

   public:
    void Calculate(const std::vector<GPUVertex>& vertices, const std::vector<GPUFace>& faces);
    const GPUBVHNode* GetGPUBVHNodes() const { return nodes.data(); }
    size_t GetNodeCount() const { return nodes_used; }
    const std::vector<uint32_t>& GetFaceIndices() const { return face_indices; }
    int GetMaxDepth() const { return max_depth; }
    // adopt a build made elsewhere (rt_bvh_build_device, byte-identical to Calculate)
    void Adopt(std::vector<GPUBVHNode> built_nodes, std::vector<uint32_t> built_face_indices, int depth);
};

// A triangle mesh as the reference receives it from assimp (aiMesh positions/normals/faces).
struct LoadedMesh {
    std::vector<float> positions;  // [n][3]
    std::vector<float> normals;    // [n][3]
    std::vector<uint32_t> indices; // [f][3]
    mat4 transform;                // node transform incl. the importer's root rotation
};
std::unique_ptr<LoadedMesh> LoadMeshAsset(const std::string& path);
// Wavefront OBJ through the reference importer's post-processing, restated (objload.cpp).
std::unique_ptr<LoadedMesh> LoadObjMesh(const std::string& path, float smoothing_angle_deg = 100.0f);
// aiMatrix4x4::RotationX(-pi/2) at the root, as utils/AssimpLoader.cpp:47-48 applies it.
mat4 ImporterRootTransform();

// Scene.h:87-129
struct Scene : public GPUScene {
    Scene();
    ~Scene();
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;

    void AddSphere(f3 position, float radius, int material = 0);
    void AddTriangle(f3 a, f3 b, f3 c, int material = 0);
    void AddQuad(f3 a, f3 b, f3 c, f3 d, int material = 0) {
        AddTriangle(a, b, c, material);
        AddTriangle(c, d, a, material);
    }
    uint32_t AddMaterial(const Material& material);
    void AddLoadedScene(const LoadedMesh& mesh, const mat4& transform, int default_material = 0);
    void SetEnvironment(const std::vector<float>& rgba_level0, int size);
    const std::vector<float>& EnvironmentTexels() const { return environment_texels; }
    int EnvironmentSize() const { return environment_size; }
    void Upload(void* rng_state);
    void BuildHost();

    Camera& GetCamera() { return camera; }
    void AddDirtyFlags(DirtyFlags flags = ~0u) { dirty_flags |= flags; }
    void AddDirtyFlag(DirtyFlagValue flag) { AddDirtyFlags(static_cast<DirtyFlags>(flag)); }
    bool IsFlagDirty(DirtyFlagValue flag) const { return dirty_flags & static_cast<DirtyFlags>(flag); }

    const std::vector<GPUVertex>& HostVertices() const { return vertices; }
    const std::vector<GPUFace>& HostFaces() const { return faces; }
    const BVH& GetBVH() const { return *bvh; }

   private:
    Camera camera;
    std::vector<GeometrySphere> spheres;
    std::vector<Material> materials;
    std::vector<GPUFace> faces;
    std::vector<GPUVertex> vertices;
    std::unique_ptr<DeviceMemory> memory, materials_memory, bvh_memory, bvh_face_index_memory, faces_memory,
        vertices_memory;
    uint64_t environment = 0;
    std::vector<float> environment_texels;
    int environment_size = 0;
    bool environment_dirty = false;
    std::unique_ptr<BVH> bvh;
    DirtyFlags dirty_flags = ~0u;
    bool bvh_upload_pending = false;
    bool tris_pending = false;
};

// CUDARayTracer::SetupCornellBox / SetupStanfordBunny (RayTracing/RayTracing.cpp:79-203, 33-69)
// and the two synthetic benchmark scenes of BASELINE.json configs 4 and 5.
void SetupCornellBox(Scene& scene);
void SetupStanfordBunny(Scene& scene, const LoadedMesh& bunny);
void SetupFourBunnies(Scene& scene, const LoadedMesh& bunny);
void SetupPlaneGrid(Scene& scene, int n);

}  // namespace RayTracing

#include "mirror.h"  // rt_internal_* mirror registry

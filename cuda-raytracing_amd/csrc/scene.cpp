// scene.cpp -- host scene construction, BVH build and upload.  Restates RayTracing/Scene.cpp,
// RayTracing/BVH.cpp and the scene setup of RayTracing/RayTracing.cpp (file:line cited per
// function) so that the arrays handed to the kernel are byte-identical to the reference's.
#include "scene.h"
#include "mirror.h"

#include <algorithm>
#include <cmath>
#include <array>
#include <cstdio>
#include <cstring>
#include <fstream>

namespace RayTracing {

using rtm::add;
using rtm::cross;
using rtm::divs;
using rtm::mk;
using rtm::muls;
using rtm::normalize;
using rtm::sub;

DeviceMemory::DeviceMemory(size_t n) : size(n) {
    if (rt_malloc(&memory, n == 0 ? 16 : n) != 0) throw std::runtime_error("allocation failed");
}
DeviceMemory::~DeviceMemory() {
    if (memory) rt_free(memory);
}

static void upload(DeviceMemory& mem, const void* src, size_t bytes) {
    if (bytes && rt_memcpy_h2d(mem.GetMemory(), src, bytes) != 0) {
        // CUDA_CHECK semantics (utils/CUDAHelper.h:8-18): print and exit.
        std::fprintf(stderr, "rt error: %s\n", rt_last_error());
        std::exit(EXIT_FAILURE);
    }
}

// ---------------------------------------------------------------------------------------
// Camera (Scene.cpp:15-36)
// ---------------------------------------------------------------------------------------
Camera::Camera() {
    std::memset(static_cast<GPUCamera*>(this), 0, sizeof(GPUCamera));
    viewport_worldspace_size[0] = viewport_worldspace_size[1] = 1.0f;
    aspect = 1.0f;
    transform = projection = view = rth::identity();
}

void Camera::Update() {
    aspect = viewport_w / viewport_h;
    // ComposeMatrix(origin, quat(vec3(radians(x), radians(y), 0)), vec3(1)) (Math.h:63-70)
    rth::quat q = rth::quat_from_euler(mk(rth::radians(angle_x), rth::radians(angle_y), 0.0f));
    mat4 t = rth::translate(rth::identity(), mk(origin[0], origin[1], origin[2]));
    t = rth::mul(t, rth::mat4_cast(q));
    transform = rth::scale(t, mk(1, 1, 1));
    projection = rth::perspective_rh_no(rth::radians(fov_y), aspect, 1.0f, 1000.0f);
    view = rth::inverse(transform);
    mat4 inv_proj = rth::inverse(projection);
    rtm::f4 ll4 = rth::mulv(inv_proj, rtm::f4{-1, -1, -1, 1});
    rtm::f4 ur4 = rth::mulv(inv_proj, rtm::f4{1, 1, -1, 1});
    f3 ll = mk(ll4.x / ll4.w, ll4.y / ll4.w, ll4.z / ll4.w);
    f3 ur = mk(ur4.x / ur4.w, ur4.y / ur4.w, ur4.z / ur4.w);
    viewport_worldspace_size[0] = ur.x - ll.x;
    viewport_worldspace_size[1] = ur.y - ll.y;
    rtm::f4 h = rth::mulv(transform, rtm::f4{viewport_worldspace_size[0], 0, 0, 0});
    rtm::f4 v = rth::mulv(transform, rtm::f4{0, viewport_worldspace_size[1], 0, 0});
    rtm::f4 l = rth::mulv(transform, rtm::f4{ll.x, ll.y, ll.z, 1});
    horizontal[0] = h.x, horizontal[1] = h.y, horizontal[2] = h.z;
    vertical[0] = v.x, vertical[1] = v.y, vertical[2] = v.z;
    lower_left_corner[0] = l.x, lower_left_corner[1] = l.y, lower_left_corner[2] = l.z;
}

// Scene.h:76-80
Material::Material(f3 a, f3 e) {
    albedo[0] = a.x, albedo[1] = a.y, albedo[2] = a.z, albedo[3] = 1.0f;
    emissive[0] = e.x, emissive[1] = e.y, emissive[2] = e.z, emissive[3] = 1.0f;
    specular[0] = specular[1] = specular[2] = specular[3] = 0.0f;
    roughness = 0.9f;
    specular_percent = 0.0f;
    IOR = 1.0f;
}

// ---------------------------------------------------------------------------------------
// BVH (BVH.cpp:8-124)
// ---------------------------------------------------------------------------------------
void BVH::Calculate(const std::vector<GPUVertex>& v, const std::vector<GPUFace>& f) {
    nodes.clear();
    triangles.clear();
    face_indices.clear();
    max_depth = 0;
    if (f.empty()) {
        nodes.resize(1);
        GPUBVHNode& root = nodes[0];
        for (int k = 0; k < 3; k++) root.bmin[k] = 1e30f, root.bmax[k] = -1e30f;
        root.first_index = root.prim_count = 0;
        nodes_used = 1;
        vertices = v.data(), faces = f.data();
        return;
    }
    GPUBVHNode blank;
    for (int k = 0; k < 3; k++) blank.bmin[k] = 1e30f, blank.bmax[k] = -1e30f;
    blank.first_index = blank.prim_count = 0;
    nodes.assign(f.size() * 2 - 1, blank);
    triangles.reserve(f.size());
    vertices = v.data();
    faces = f.data();
    for (uint32_t i = 0; i < f.size(); i++) {
        const float* p0 = vertices[faces[i].v0].position;
        const float* p1 = vertices[faces[i].v1].position;
        const float* p2 = vertices[faces[i].v2].position;
        Triangle t;
        t.centroid = divs(add(add(mk(p0[0], p0[1], p0[2]), mk(p1[0], p1[1], p1[2])), mk(p2[0], p2[1], p2[2])), 3.0f);
        t.index = i;
        triangles.push_back(t);
    }
    nodes_used = 1;
    GPUBVHNode& root = nodes[root_node_id];
    root.first_index = 0;
    root.prim_count = (uint32_t)f.size();
    UpdateBounds(root_node_id);
    Subdivide(root_node_id, 0);
    face_indices.resize(f.size());
    for (size_t i = 0; i < triangles.size(); i++) face_indices[i] = triangles[i].index;
}

void BVH::Adopt(std::vector<GPUBVHNode> built_nodes, std::vector<uint32_t> built_face_indices, int depth) {
    nodes = std::move(built_nodes);
    nodes_used = (uint32_t)nodes.size();
    face_indices = std::move(built_face_indices);
    triangles.clear();
    max_depth = depth;
}

void BVH::UpdateBounds(uint32_t node_index) {
    GPUBVHNode& node = nodes.at(node_index);
    for (int k = 0; k < 3; k++) node.bmin[k] = 1e30f, node.bmax[k] = -1e30f;
    for (uint32_t i = 0; i < node.prim_count; i++) {
        const Triangle& t = triangles.at(node.first_index + i);
        const uint32_t vi[3] = {faces[t.index].v0, faces[t.index].v1, faces[t.index].v2};
        for (uint32_t idx : vi) {
            const float* p = vertices[idx].position;
            for (int k = 0; k < 3; k++) {
                node.bmin[k] = rtm::gmin(node.bmin[k], p[k]);
                node.bmax[k] = rtm::gmax(node.bmax[k], p[k]);
            }
        }
    }
}

static inline float comp(const f3& v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

void BVH::Subdivide(uint32_t node_index, int depth) {
    if (depth > max_depth) max_depth = depth;
    GPUBVHNode& node = nodes.at(node_index);
    const float extent[3] = {node.bmax[0] - node.bmin[0], node.bmax[1] - node.bmin[1], node.bmax[2] - node.bmin[2]};
    int axis1 = 0;
    if (extent[1] > extent[0]) axis1 = 1;
    if (extent[2] > extent[axis1]) axis1 = 2;
    int axis2 = (axis1 + 1) % 3;
    int axis3 = (axis2 + 1) % 3;
    if (extent[axis3] > extent[axis2]) std::swap(axis2, axis3);
    const std::array<int, 3> try_axis = {axis1, axis2, axis3};

    bool found = false;
    int i = 0;
    int left_count = 0;
    for (int axis : try_axis) {
        const float split_pos = node.bmin[axis] + extent[axis] * 0.5f;
        i = (int)node.first_index;
        int j = i + (int)node.prim_count - 1;
        while (i <= j) {
            if (comp(triangles[i].centroid, axis) < split_pos)
                i++;
            else
                std::swap(triangles[i], triangles[j--]);
        }
        left_count = i - (int)node.first_index;
        const bool left_empty = left_count == 0;
        const bool right_empty = left_count == (int)node.prim_count;
        if (!left_empty && !right_empty) {
            found = true;
            break;
        }
    }
    if (!found) return;

    const int left = (int)nodes_used++;
    const int right = (int)nodes_used++;
    nodes[left].first_index = node.first_index;
    node.first_index = (uint32_t)left;
    nodes[left].prim_count = (uint32_t)left_count;
    nodes[right].first_index = (uint32_t)i;
    nodes[right].prim_count = node.prim_count - (uint32_t)left_count;
    node.prim_count = 0;
    UpdateBounds(left);
    UpdateBounds(right);
    Subdivide(left, depth + 1);
    Subdivide(right, depth + 1);
}

// ---------------------------------------------------------------------------------------
// Scene (Scene.cpp)
// ---------------------------------------------------------------------------------------
Scene::Scene() {
    std::memset(static_cast<GPUScene*>(this), 0, sizeof(GPUScene));
    bvh = std::make_unique<BVH>();
}
Scene::~Scene() {
    if (gpu_bvh_nodes) rt_internal_forget_mirror(gpu_bvh_nodes);
    if (environment) rt_cubemap_destroy(environment);
}

// Scene.cpp:46-67.  Note GPUFace{index0, index0+1, index0+2} fills v0, v2, v1 in that order.
void Scene::AddTriangle(f3 a, f3 b, f3 c, int material) {
    const f3 n = normalize(cross(sub(c, b), sub(a, b)));
    const uint32_t index0 = (uint32_t)vertices.size();
    const f3 p[3] = {a, b, c};
    for (const f3& q : p) {
        GPUVertex v;
        v.position[0] = q.x, v.position[1] = q.y, v.position[2] = q.z;
        v.normal[0] = n.x, v.normal[1] = n.y, v.normal[2] = n.z;
        v.uv[0] = v.uv[1] = 0.0f;
        vertices.push_back(v);
    }
    GPUFace face;
    face.v0 = index0;
    face.v2 = index0 + 1;
    face.v1 = index0 + 2;
    face.material = (uint32_t)material;
    faces.push_back(face);
    AddDirtyFlag(DirtyFlagValue::SceneMemory);
}

// Scene.cpp:69-73
void Scene::AddSphere(f3 position, float radius, int material) {
    GeometrySphere s;
    std::memset(&s, 0, sizeof(s));
    s.position[0] = position.x, s.position[1] = position.y, s.position[2] = position.z;
    s.radius = radius;
    s.material = material;
    spheres.push_back(s);
    AddDirtyFlag(DirtyFlagValue::SceneMemory);
}

// Scene.cpp:134-139
uint32_t Scene::AddMaterial(const Material& material) {
    AddDirtyFlag(DirtyFlagValue::SceneMemory);
    materials.push_back(material);
    return (uint32_t)materials.size() - 1;
}

// Scene.cpp:75-132: indexed smooth faces + a flat duplicate of every face via AddTriangle.
void Scene::AddLoadedScene(const LoadedMesh& mesh, const mat4& transform, int default_material) {
    AddDirtyFlag(DirtyFlagValue::BVH);
    AddDirtyFlag(DirtyFlagValue::SceneMemory);
    const uint32_t index_offset = (uint32_t)vertices.size();
    const mat4 mt = rth::mul(transform, mesh.transform);
    const size_t nv = mesh.positions.size() / 3;
    auto xform_pos = [&](uint32_t i) {
        rtm::f4 p = rth::mulv(mt, rtm::f4{mesh.positions[3 * i], mesh.positions[3 * i + 1], mesh.positions[3 * i + 2], 1.0f});
        return mk(p.x, p.y, p.z);
    };
    for (uint32_t v = 0; v < nv; v++) {
        GPUVertex vert;
        f3 p = xform_pos(v);
        rtm::f4 n = rth::mulv(mt, rtm::f4{mesh.normals[3 * v], mesh.normals[3 * v + 1], mesh.normals[3 * v + 2], 0.0f});
        vert.position[0] = p.x, vert.position[1] = p.y, vert.position[2] = p.z;
        vert.normal[0] = n.x, vert.normal[1] = n.y, vert.normal[2] = n.z;
        vert.uv[0] = vert.uv[1] = 0.0f;  // HasTextureCoords(0) is false for the bunny
        vertices.push_back(vert);
    }
    const size_t nf = mesh.indices.size() / 3;
    for (size_t f = 0; f < nf; f++) {
        const uint32_t* idx = &mesh.indices[3 * f];
        GPUFace face;
        face.v0 = idx[0] + index_offset;
        face.v1 = idx[1] + index_offset;
        face.v2 = idx[2] + index_offset;
        face.material = (uint32_t)default_material;
        faces.push_back(face);
        AddTriangle(xform_pos(idx[0]), xform_pos(idx[1]), xform_pos(idx[2]), default_material);
    }
}

// Scene::Scene loads the sky at construction (Scene.cpp:38-41); here the texels are kept on
// the host and the device cube map is created by the next Upload.
void Scene::SetEnvironment(const std::vector<float>& rgba, int size) {
    environment_texels = rgba;
    environment_size = size;
    environment_dirty = true;
}

// The host half of Scene::Upload (Scene.cpp:182-199): camera basis + BVH build when dirty.
void Scene::BuildHost() {
    camera.Update();
    if (IsFlagDirty(DirtyFlagValue::BVH)) {
        bvh->Calculate(vertices, faces);
        dirty_flags &= ~static_cast<DirtyFlags>(DirtyFlagValue::BVH);
        bvh_upload_pending = true;
    }
}

// Geometry at least this large builds its BVH on the GPU (rt_bvh_build_device, byte-identical to
// BVH::Calculate; 4-7x faster on the BASELINE scenes); rt_build_options.host_bvh keeps the host builder.
static constexpr size_t kGpuBvhMinFaces = 65536;

// Scene.cpp:182-234
void Scene::Upload(void* rng) {
    rt_build_options opt;
    rt_get_build_options(&opt);
    const bool host_bvh = opt.host_bvh != 0;
    bool gpu_bvh = IsFlagDirty(DirtyFlagValue::BVH) && faces.size() >= kGpuBvhMinFaces && !host_bvh;
    if (gpu_bvh) {
        // vertices and faces first, then the build reads them on the device
        const size_t nv = vertices.size() * sizeof(GPUVertex), nf = faces.size() * sizeof(GPUFace);
        vertices_memory = std::make_unique<DeviceMemory>(nv);
        gpu_vertices = (const GPUVertex*)vertices_memory->GetMemory();
        upload(*vertices_memory, vertices.data(), nv);
        faces_memory = std::make_unique<DeviceMemory>(nf);
        gpu_faces = (const GPUFace*)faces_memory->GetMemory();
        upload(*faces_memory, faces.data(), nf);
        if (gpu_bvh_nodes) rt_internal_forget_mirror(gpu_bvh_nodes);
        const uint32_t n = (uint32_t)faces.size();
        auto nodes_mem = std::make_unique<DeviceMemory>((2 * (size_t)n - 1) * sizeof(GPUBVHNode));
        auto fi_mem = std::make_unique<DeviceMemory>((size_t)n * sizeof(uint32_t));
        uint32_t count = 0;
        int depth = 0;
        if (rt_bvh_build_device(gpu_vertices, (uint32_t)vertices.size(), gpu_faces, n, (GPUBVHNode*)nodes_mem->GetMemory(),
                                (uint32_t*)fi_mem->GetMemory(), &count, &depth, nullptr) == 0) {
            bvh_memory = std::move(nodes_mem);
            bvh_face_index_memory = std::move(fi_mem);
            gpu_bvh_nodes = (const GPUBVHNode*)bvh_memory->GetMemory();
            gpu_bvh_face_indices = (const uint32_t*)bvh_face_index_memory->GetMemory();
            // the host keeps a copy (mirror, diagnostics), as after BVH::Calculate
            std::vector<GPUBVHNode> hn(count);
            std::vector<uint32_t> hf(n);
            if (rt_memcpy_d2h(hn.data(), gpu_bvh_nodes, count * sizeof(GPUBVHNode)) != 0 ||
                rt_memcpy_d2h(hf.data(), gpu_bvh_face_indices, n * sizeof(uint32_t)) != 0)
                throw std::runtime_error(rt_last_error());
            bvh->Adopt(std::move(hn), std::move(hf), depth);
            dirty_flags &= ~static_cast<DirtyFlags>(DirtyFlagValue::BVH);
            tris_pending = true;
        }
        // otherwise (e.g. non-finite vertex positions) the host builder below handles the input
    }
    BuildHost();  // camera.Update() + BVH::Calculate when dirty
    static_cast<GPUScene*>(this)->camera = static_cast<const GPUCamera&>(camera);
    rng_state = rng;
    if (environment_dirty) {
        if (environment) rt_cubemap_destroy(environment);
        environment = rt_cubemap_create(environment_texels.data(), environment_size);
        if (!environment) throw std::runtime_error(rt_last_error());
        environment_dirty = false;
    }
    environment_cubemap_tex = environment;

    if (bvh_upload_pending || IsFlagDirty(DirtyFlagValue::SceneMemory)) tris_pending = true;
    if (bvh_upload_pending) {
        bvh_upload_pending = false;
        if (gpu_bvh_nodes) rt_internal_forget_mirror(gpu_bvh_nodes);
        const size_t nb = bvh->GetNodeCount() * sizeof(GPUBVHNode);
        bvh_memory = std::make_unique<DeviceMemory>(nb);
        gpu_bvh_nodes = (const GPUBVHNode*)bvh_memory->GetMemory();
        upload(*bvh_memory, bvh->GetGPUBVHNodes(), nb);
        const size_t ni = bvh->GetFaceIndices().size() * sizeof(uint32_t);
        bvh_face_index_memory = std::make_unique<DeviceMemory>(ni);
        gpu_bvh_face_indices = (const uint32_t*)bvh_face_index_memory->GetMemory();
        upload(*bvh_face_index_memory, bvh->GetFaceIndices().data(), ni);
    }
    if (IsFlagDirty(DirtyFlagValue::SceneMemory)) {
        const size_t ns = spheres.size() * sizeof(GeometrySphere);
        if (!memory || memory->GetSize() < ns) memory = std::make_unique<DeviceMemory>(ns);
        sphere_count = (int)spheres.size();
        gpu_spheres = (const GeometrySphere*)memory->GetMemory();
        upload(*memory, spheres.data(), ns);
        const size_t nm = materials.size() * sizeof(GPUMaterial);
        std::vector<GPUMaterial> gm(materials.begin(), materials.end());
        materials_memory = std::make_unique<DeviceMemory>(nm);
        material_count = (int)materials.size();
        upload(*materials_memory, gm.data(), nm);
        gpu_materials = (const GPUMaterial*)materials_memory->GetMemory();
        if (!gpu_bvh) {  // (already uploaded for the GPU build)
            const size_t nv = vertices.size() * sizeof(GPUVertex);
            vertices_memory = std::make_unique<DeviceMemory>(nv);
            gpu_vertices = (const GPUVertex*)vertices_memory->GetMemory();
            upload(*vertices_memory, vertices.data(), nv);
            const size_t nf = faces.size() * sizeof(GPUFace);
            faces_memory = std::make_unique<DeviceMemory>(nf);
            gpu_faces = (const GPUFace*)faces_memory->GetMemory();
            upload(*faces_memory, faces.data(), nf);
        }
    }
    if (tris_pending) {
        // the kernel's private triangle mirror (mirror.h), built from the arrays just uploaded
        MirrorHost m;
        const std::vector<uint32_t>& fi = bvh->GetFaceIndices();
        rt_build_mirror(bvh->GetGPUBVHNodes(), bvh->GetNodeCount(), fi.data(), fi.size(), faces.data(), faces.size(),
                        vertices.data(), vertices.size(), &m);
        if (rt_internal_install_mirror(this, m) != 0) throw std::runtime_error(rt_last_error());
        tris_pending = false;
    }
    dirty_flags = 0;
}

// ---------------------------------------------------------------------------------------
// Assets
// ---------------------------------------------------------------------------------------
// assimp aiMatrix4x4 (row-major) helpers for the importer's root rotation
// (utils/AssimpLoader.cpp:8-27,47-48).
struct AiMat {
    float r[4][4];  // r[row][col]
};
static AiMat ai_identity() {
    AiMat m;
    std::memset(&m, 0, sizeof(m));
    for (int i = 0; i < 4; i++) m.r[i][i] = 1.0f;
    return m;
}
// aiMatrix4x4t::operator*= : this(r,c) = m(0,c)*this(r,0) + m(1,c)*this(r,1) + m(2,c)*this(r,2) + m(3,c)*this(r,3)
static AiMat ai_mul(const AiMat& a, const AiMat& m) {
    AiMat o;
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++)
            o.r[r][c] = ((m.r[0][c] * a.r[r][0] + m.r[1][c] * a.r[r][1]) + m.r[2][c] * a.r[r][2]) + m.r[3][c] * a.r[r][3];
    return o;
}

// aiMatrix4x4::RotationX(-(float)M_PI / 2) as the accumulated root transform, times the
// (identity) root and mesh node transforms, then convert_matrix (transpose into glm).
mat4 ImporterRootTransform() {
    const float a = -3.14159265358979323846f / 2;
    AiMat rx = ai_identity();
    rx.r[1][1] = rx.r[2][2] = rth::hcos(a);
    rx.r[2][1] = rth::hsin(a);
    rx.r[1][2] = -rx.r[2][1];
    const AiMat acc = ai_mul(ai_mul(rx, ai_identity()), ai_identity());
    mat4 t;
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) t.m[c][r] = acc.r[r][c];
    return t;
}

std::unique_ptr<LoadedMesh> LoadMeshAsset(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return nullptr;
    char magic[8];
    uint32_t nv = 0, nf = 0;
    in.read(magic, 8);
    in.read(reinterpret_cast<char*>(&nv), 4);
    in.read(reinterpret_cast<char*>(&nf), 4);
    if (!in || std::memcmp(magic, "RTMESH01", 8) != 0) return nullptr;
    auto mesh = std::make_unique<LoadedMesh>();
    mesh->positions.resize((size_t)nv * 3);
    mesh->normals.resize((size_t)nv * 3);
    mesh->indices.resize((size_t)nf * 3);
    in.read(reinterpret_cast<char*>(mesh->positions.data()), (std::streamsize)nv * 12);
    in.read(reinterpret_cast<char*>(mesh->normals.data()), (std::streamsize)nv * 12);
    in.read(reinterpret_cast<char*>(mesh->indices.data()), (std::streamsize)nf * 12);
    if (!in) return nullptr;
    mesh->transform = ImporterRootTransform();
    return mesh;
}

static bool load_cube(const std::string& path, std::vector<float>& rgba, int& size) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    std::vector<char> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    if (buf.size() >= 12 && std::memcmp(buf.data(), "RTCUBE01", 8) == 0) {
        uint32_t s;
        std::memcpy(&s, buf.data() + 8, 4);
        const size_t n = (size_t)6 * s * s * 4;
        if (buf.size() < 12 + n * 4) return false;
        rgba.resize(n);
        std::memcpy(rgba.data(), buf.data() + 12, n * 4);
        size = (int)s;
        return true;
    }
    // Legacy DDS cube map, fp32 RGBA (D3DFMT 116): utils/image/DDSLoader.cpp:135-371 slices the
    // face-major file (all mips of face 0, then face 1, ...); level 0 of each face is used.
    if (buf.size() < 128 || std::memcmp(buf.data(), "DDS ", 4) != 0) return false;
    uint32_t h[31];
    std::memcpy(h, buf.data() + 4, sizeof(h));
    const uint32_t height = h[2], width = h[3], mips = h[6] ? h[6] : 1, pf_flags = h[19], fourcc = h[20],
                   caps2 = h[27];
    if (h[0] != 124 || width != height || !(pf_flags & 4) || fourcc != 116 || (caps2 & 0xFE00) != 0xFE00) return false;
    size_t face_bytes = 0;
    for (uint32_t m = 0; m < mips; m++) face_bytes += (size_t)16 * (width >> m) * (height >> m);
    if (buf.size() < 128 + 6 * face_bytes) return false;
    rgba.resize((size_t)6 * width * width * 4);
    for (int f = 0; f < 6; f++)
        std::memcpy(rgba.data() + (size_t)f * width * width * 4, buf.data() + 128 + f * face_bytes,
                    (size_t)16 * width * width);
    size = (int)width;
    return true;
}

// ---------------------------------------------------------------------------------------
// Scene setups (RayTracing.cpp:79-203 and 33-69)
// ---------------------------------------------------------------------------------------
static Material mat_spec(f3 albedo, float spec_pct, f3 spec, float rough) {
    Material m(albedo);
    m.specular_percent = spec_pct;
    m.specular[0] = spec.x, m.specular[1] = spec.y, m.specular[2] = spec.z, m.specular[3] = 0.0f;
    m.roughness = rough;
    return m;
}

void SetupCornellBox(Scene& s) {
    const f3 gray = mk(0.7f, 0.7f, 0.7f), black = mk(0, 0, 0);
    {  // back wall
        int m = (int)s.AddMaterial(Material(gray, black));
        s.AddQuad(mk(-12.6f, -12.6f, 25.0f), mk(12.6f, -12.6f, 25.0f), mk(12.6f, 12.6f, 25.0f), mk(-12.6f, 12.6f, 25.0f), m);
    }
    {  // floor
        int m = (int)s.AddMaterial(Material(gray, black));
        s.AddQuad(mk(-12.6f, -12.45f, 25.0f), mk(12.6f, -12.45f, 25.0f), mk(12.6f, -12.45f, 15.0f), mk(-12.6f, -12.45f, 15.0f), m);
    }
    {  // ceiling
        int m = (int)s.AddMaterial(Material(gray, black));
        s.AddQuad(mk(-12.6f, 12.5f, 25.0f), mk(12.6f, 12.5f, 25.0f), mk(12.6f, 12.5f, 15.0f), mk(-12.6f, 12.5f, 15.0f), m);
    }
    {  // left wall
        int m = (int)s.AddMaterial(Material(mk(0.1f, 0.7f, 0.1f), black));
        s.AddQuad(mk(-12.5f, -12.6f, 25.0f), mk(-12.5f, -12.6f, 15.0f), mk(-12.5f, 12.6f, 15.0f), mk(-12.5f, 12.6f, 25.0f), m);
    }
    {  // right wall
        int m = (int)s.AddMaterial(Material(mk(0.7f, 0.1f, 0.1f), black));
        s.AddQuad(mk(12.5f, -12.6f, 25.0f), mk(12.5f, -12.6f, 15.0f), mk(12.5f, 12.6f, 15.0f), mk(12.5f, 12.6f, 25.0f), m);
    }
    {  // light
        int m = (int)s.AddMaterial(Material(black, muls(mk(1.0f, 0.9f, 0.7f), 20.0f)));
        s.AddQuad(mk(-5.0f, 12.4f, 22.5f), mk(5.0f, 12.4f, 22.5f), mk(5.0f, 12.4f, 17.5f), mk(-5.0f, 12.4f, 17.5f), m);
    }
    const f3 white9 = mk(0.9f, 0.9f, 0.9f);
    s.AddSphere(mk(-9.0f, -9.5f, 20.0f), 3, (int)s.AddMaterial(mat_spec(mk(0.9f, 0.9f, 0.50f), 0.5f, white9, 0.2f)));
    s.AddSphere(mk(0.0f, -9.5f, 20.0f), 3, (int)s.AddMaterial(mat_spec(mk(0.9f, 0.5f, 0.90f), 0.3f, white9, 0.2f)));
    s.AddSphere(mk(9.0f, -9.5f, 20.0f), 3, (int)s.AddMaterial(mat_spec(mk(0.0f, 0.0f, 1.0f), 0.5f, mk(1.0f, 0.0f, 0.0f), 0.4f)));
    s.GetCamera().SetYAndle(180);
    // shiny green balls of varying roughness
    const f3 green = mk(0.3f, 1.0f, 0.3f), one = mk(1, 1, 1);
    const float xs[5] = {-10.0f, -5.0f, 0.0f, 5.0f, 10.0f};
    const float rs[5] = {0.0f, 0.25f, 0.5f, 0.75f, 0.97f};
    for (int i = 0; i < 5; i++) s.AddSphere(mk(xs[i], 0.0f, 23.0f), 1.75f, (int)s.AddMaterial(mat_spec(one, 1.0f, green, rs[i])));
}

static mat4 bunny_transform(f3 translation) {
    mat4 m = rth::translate(rth::identity(), translation);
    m = rth::rotate(m, -3.14159265358979323846f, mk(0, 1, 0));
    m = rth::rotate(m, 3.14159265358979323846f / 2, mk(1, 0, 0));
    return rth::scale(m, mk(150.0f, 150.0f, 150.0f));
}

static void bunny_floor_and_light(Scene& s) {
    {
        const f3 offset = mk(20, 0, 0), sc = mk(50, 1, 50);
        f3 A = add(rtm::mul(sc, mk(-1.0f, -12.45f, 1.0f)), offset);
        f3 B = add(rtm::mul(sc, mk(1.0f, -12.45f, 1.0f)), offset);
        f3 C = add(rtm::mul(sc, mk(1.0f, -12.45f, -1.0f)), offset);
        f3 D = add(rtm::mul(sc, mk(-1.0f, -12.45f, -1.0f)), offset);
        int m = (int)s.AddMaterial(Material(mk(0.7f, 0.7f, 0.7f), mk(0.0f, 0.0f, 0.0f)));
        s.AddQuad(A, B, C, D, m);
    }
    {
        int m = (int)s.AddMaterial(Material(mk(0, 0, 0), muls(mk(0.3f, 0.9f, 0.7f), 10.0f)));
        s.AddSphere(mk(30, 10, 40), 8, m);
    }
}

void SetupStanfordBunny(Scene& s, const LoadedMesh& bunny) {
    const int m = (int)s.AddMaterial(mat_spec(mk(1, 1, 1), 0.5f, mk(0.3f, 1.0f, 0.3f), 0.8f));
    s.AddLoadedScene(bunny, bunny_transform(mk(30, -18, 20)), m);
    bunny_floor_and_light(s);
}

// BASELINE.json config 4: four bunnies with the reference rotation/scale.
void SetupFourBunnies(Scene& s, const LoadedMesh& bunny) {
    const int m = (int)s.AddMaterial(mat_spec(mk(1, 1, 1), 0.5f, mk(0.3f, 1.0f, 0.3f), 0.8f));
    const f3 t[4] = {mk(17, -18, 7), mk(43, -18, 7), mk(17, -18, 33), mk(43, -18, 33)};
    for (const f3& tr : t) s.AddLoadedScene(bunny, bunny_transform(tr), m);
    bunny_floor_and_light(s);
}

// BASELINE.json config 5: an n x n quad grid on z = 30, x in [-60, 60], y in [-34, 34]
// (2 n^2 triangles; n = 708 gives 1,002,528), facing the default camera.
void SetupPlaneGrid(Scene& s, int n) {
    const int m = (int)s.AddMaterial(Material(mk(0.7f, 0.7f, 0.7f), mk(0.2f, 0.2f, 0.2f)));
    std::vector<float> xs(n + 1), ys(n + 1);
    for (int i = 0; i <= n; i++) {
        xs[i] = -60.0f + 120.0f * (float)i / (float)n;
        ys[i] = -34.0f + 68.0f * (float)i / (float)n;
    }
    for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++)
            s.AddQuad(mk(xs[i], ys[j], 30.0f), mk(xs[i + 1], ys[j], 30.0f), mk(xs[i + 1], ys[j + 1], 30.0f),
                      mk(xs[i], ys[j + 1], 30.0f), m);
    s.GetCamera().SetYAndle(180);
    s.AddDirtyFlag(DirtyFlagValue::BVH);
}

}  // namespace RayTracing

// ---------------------------------------------------------------------------------------
// C-ABI wrappers (include/rt_abi.h)
// ---------------------------------------------------------------------------------------
using RayTracing::Scene;

struct rt_scene {
    Scene scene;
};

static rtm::f3 v3(const float* p) { return rtm::f3{p[0], p[1], p[2]}; }

extern "C" {

rt_scene* rt_scene_create(void) {
    try {
        return new rt_scene();
    } catch (...) {
        return nullptr;
    }
}
void rt_scene_destroy(rt_scene* s) { delete s; }

uint32_t rt_scene_add_material(rt_scene* s, const GPUMaterial* m) {
    RayTracing::Material mat;
    static_cast<GPUMaterial&>(mat) = *m;
    return s->scene.AddMaterial(mat);
}
void rt_scene_add_triangle(rt_scene* s, const float a[3], const float b[3], const float c[3], int material) {
    s->scene.AddTriangle(v3(a), v3(b), v3(c), material);
    s->scene.AddDirtyFlag(RayTracing::DirtyFlagValue::BVH);
}
void rt_scene_add_quad(rt_scene* s, const float a[3], const float b[3], const float c[3], const float d[3],
                       int material) {
    s->scene.AddQuad(v3(a), v3(b), v3(c), v3(d), material);
    s->scene.AddDirtyFlag(RayTracing::DirtyFlagValue::BVH);
}
void rt_scene_add_sphere(rt_scene* s, const float p[3], float radius, int material) {
    s->scene.AddSphere(v3(p), radius, material);
}
int rt_scene_add_mesh_file(rt_scene* s, const char* path, const float transform[16], int material) {
    const std::string p(path);
    const bool obj = p.size() > 4 && (p.compare(p.size() - 4, 4, ".obj") == 0 || p.compare(p.size() - 4, 4, ".OBJ") == 0);
    auto mesh = obj ? RayTracing::LoadObjMesh(p) : RayTracing::LoadMeshAsset(p);
    if (!mesh) return 1;
    rth::mat4 t;
    std::memcpy(t.m, transform, sizeof(t.m));
    s->scene.AddLoadedScene(*mesh, t, material);
    return 0;
}
int rt_scene_set_environment_file(rt_scene* s, const char* path) {
    std::vector<float> rgba;
    int size = 0;
    if (!RayTracing::load_cube(path, rgba, size)) return 1;
    s->scene.SetEnvironment(rgba, size);
    return 0;
}
int rt_scene_environment(const rt_scene* s, const float** texels, int* size) {
    if (!s || !texels || !size) return 1;
    const auto& t = s->scene.EnvironmentTexels();
    *texels = t.empty() ? nullptr : t.data();
    *size = s->scene.EnvironmentSize();
    return 0;
}
void rt_scene_set_camera(rt_scene* s, const float p[3], float ax, float ay) {
    s->scene.GetCamera().SetPosition(v3(p));
    s->scene.GetCamera().SetXAndle(ax);
    s->scene.GetCamera().SetYAndle(ay);
}
void rt_scene_set_viewport(rt_scene* s, int w, int h) { s->scene.GetCamera().SetViewportSize((float)w, (float)h); }
int rt_scene_upload(rt_scene* s, void* rng_state) {
    try {
        s->scene.Upload(rng_state);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "rt_scene_upload: %s\n", e.what());
        return 1;
    }
    return 0;
}
const GPUScene* rt_scene_gpu(const rt_scene* s) { return &s->scene; }

static int host_mirror(rt_scene* s, MirrorHost* m) {
    try {
        s->scene.BuildHost();
        const auto& bvh = s->scene.GetBVH();
        const auto& fi = bvh.GetFaceIndices();
        rt_build_mirror(bvh.GetGPUBVHNodes(), bvh.GetNodeCount(), fi.data(), fi.size(), s->scene.HostFaces().data(),
                        s->scene.HostFaces().size(), s->scene.HostVertices().data(), s->scene.HostVertices().size(), m);
    } catch (const std::exception& e) {
        rt_internal_set_error(e.what());
        return -1;
    }
    return 0;
}
int rt_scene_mirror_info(rt_scene* s, size_t* tri_records, size_t* tree_nodes, size_t* tree_tri_records) {
    MirrorHost m;
    if (host_mirror(s, &m) != 0) return -1;
    *tri_records = m.tris.size() / 12;
    *tree_nodes = m.tree.size() / 16;
    *tree_tri_records = m.ltris.size() / 12;
    return 0;
}
int rt_scene_mirror_copy(rt_scene* s, float* tris, float* tree, float* tree_tris) {
    MirrorHost m;
    if (host_mirror(s, &m) != 0) return -1;
    std::copy(m.tris.begin(), m.tris.end(), tris);
    std::copy(m.tree.begin(), m.tree.end(), tree);
    std::copy(m.ltris.begin(), m.ltris.end(), tree_tris);
    return 0;
}
int rt_scene_mirror_nodes(rt_scene* s, GPUBVHNode* nodes, size_t* count) {
    MirrorHost m;
    if (host_mirror(s, &m) != 0) return -1;
    *count = m.nodes.size() / 8;
    if (nodes) std::memcpy(nodes, m.nodes.data(), m.nodes.size() * 4);
    return 0;
}
int rt_scene_mirror_twins(rt_scene* s, float* quads, size_t* quad_count, float* units, size_t* unit_count) {
    MirrorHost m;
    if (host_mirror(s, &m) != 0) return -1;
    *quad_count = m.quads.size() / 28;
    *unit_count = m.units.size() / 16;
    if (quads) std::memcpy(quads, m.quads.data(), m.quads.size() * 4);
    if (units) std::memcpy(units, m.units.data(), m.units.size() * 4);
    return 0;
}
int rt_scene_mirror_face_leaf(rt_scene* s, uint32_t* leaf, size_t* count) {
    MirrorHost m;
    if (host_mirror(s, &m) != 0) return -1;
    *count = m.face_leaf.size();
    if (leaf) std::memcpy(leaf, m.face_leaf.data(), m.face_leaf.size() * 4);
    return 0;
}
void rt_scene_build(rt_scene* s) { s->scene.BuildHost(); }
void rt_scene_camera(const rt_scene* s, GPUCamera* out) {
    *out = static_cast<const GPUCamera&>(const_cast<Scene&>(s->scene).GetCamera());
}

int rt_scene_setup(rt_scene* s, int which, const char* assets_dir) {
    const std::string dir = assets_dir ? assets_dir : "assets";
    if (which == 2) {
        RayTracing::SetupPlaneGrid(s->scene, 708);
    } else {
        auto bunny = RayTracing::LoadMeshAsset(dir + "/bunny_mesh.bin");
        if (!bunny) return 1;
        RayTracing::SetupCornellBox(s->scene);
        if (which == 0)
            RayTracing::SetupStanfordBunny(s->scene, *bunny);
        else
            RayTracing::SetupFourBunnies(s->scene, *bunny);
    }
    return rt_scene_set_environment_file(s, (dir + "/sunset_cube128.bin").c_str()) ? 2 : 0;
}

int rt_scene_setup_plane(rt_scene* s, int n, const char* assets_dir) {
    if (n <= 0) return 1;
    RayTracing::SetupPlaneGrid(s->scene, n);
    const std::string dir = assets_dir ? assets_dir : "assets";
    return rt_scene_set_environment_file(s, (dir + "/sunset_cube128.bin").c_str()) ? 2 : 0;
}

size_t rt_scene_host_arrays(const rt_scene* s, const GPUBVHNode** nodes, size_t* node_count,
                            const uint32_t** face_indices, size_t* face_count, const GPUVertex** vertices,
                            size_t* vertex_count, const GPUFace** faces) {
    const auto& bvh = s->scene.GetBVH();
    if (nodes) *nodes = bvh.GetGPUBVHNodes();
    if (node_count) *node_count = bvh.GetNodeCount();
    if (face_indices) *face_indices = bvh.GetFaceIndices().data();
    if (face_count) *face_count = s->scene.HostFaces().size();
    if (vertices) *vertices = s->scene.HostVertices().data();
    if (vertex_count) *vertex_count = s->scene.HostVertices().size();
    if (faces) *faces = s->scene.HostFaces().data();
    return bvh.GetNodeCount();
}
int rt_scene_bvh_max_depth(const rt_scene* s) { return s->scene.GetBVH().GetMaxDepth(); }

}  // extern "C"

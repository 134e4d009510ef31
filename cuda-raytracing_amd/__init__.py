"""Python host binding of the MI355X ray tracer (librt_hip.so, C-ABI in include/rt_abi.h).

Mirrors the reference's host interface so a host written against it reads the same:

* ``Scene``      -- RayTracing::Scene (RayTracing/Scene.h:87-129): AddTriangle/AddQuad/
                    AddSphere/AddMaterial/AddLoadedScene, the camera, ``upload``.
* ``RayTracer``  -- CUDARayTracer (RayTracing/RayTracing.{h,cpp}): owns the scene, the
                    per-pixel RNG state and the progressive frame index; ``process()``
                    renders one frame (RayTracing.cpp:205-234).
* ``raytracing_process`` / ``init_rng`` -- the two extern "C" entry points
                    (main_raytracing.cu:202, Random.cu:10).

Device buffers are torch tensors on the current HIP device (torch is plumbing here: memory,
streams, torch.distributed); every kernel is in librt_hip.so.  There is no CPU fallback: if
the native library is missing or fails to load this module raises.
"""
import ctypes
import os

import numpy as np
import torch  # imported before the library so librt_hip.so binds to the HIP runtime torch already loaded

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "librt_hip.so")
EXP_LIB_PATH = os.path.join(PKG_DIR, "librt_hip_exp.so")  # experimental render paths (A/B + their tests)
ASSETS_DIR = os.path.join(ROOT_DIR, "assets")

RT_RENDER_STATS = 1
RT_RENDER_VALIDATE = 16
TRACERS = {"fast": 0, "ref": 2, "flat": 4, "wavefront": 8}  # rt_render_params.flags
STAT_NAMES = ("segments", "nodes", "tri_tests", "tri_accepts", "sphere_accepts", "hits", "misses", "cycles_tree_cut",
              "wave_small_iters", "lane_small", "wave_big_tris", "lane_big_tris", "wave_segment_iters",
              "lane_segments", "tree_nodes", "tree_tri_tests", "cycles_small", "cycles_big", "cycles_total",
              "rounds_coop", "rounds_shared", "coop_rays", "cycles_tree_clusters", "cycles_tree_tris",
              "big_tests", "twin_decided", "twin_tests", "wave_big_iters", "defer_end2", "defer_redo", None, None)
STAT_COUNT = len(STAT_NAMES)  # RT_STAT_COUNT (include/rt_abi.h): per-wave records of RT_TUNE bit 11 follow
SCENES = {"bunny": 0, "bunny4": 1, "plane1m": 2}

REFERENCE_SPP = 5      # main_raytracing.cu:166-170 (Release)
REFERENCE_BOUNCES = 6  # main_raytracing.cu:115
RNG_STATE_BYTES = 48   # sizeof(curandState)


class GPUCamera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("viewport_worldspace_size", ctypes.c_float * 2),
                ("aspect", ctypes.c_float), ("horizontal", ctypes.c_float * 3),
                ("vertical", ctypes.c_float * 3), ("lower_left_corner", ctypes.c_float * 3)]


class GPUScene(ctypes.Structure):
    _fields_ = [("gpu_spheres", ctypes.c_void_p), ("gpu_materials", ctypes.c_void_p),
                ("gpu_bvh_nodes", ctypes.c_void_p), ("gpu_bvh_face_indices", ctypes.c_void_p),
                ("gpu_vertices", ctypes.c_void_p), ("gpu_faces", ctypes.c_void_p),
                ("sphere_count", ctypes.c_int32), ("material_count", ctypes.c_int32),
                ("rng_state", ctypes.c_void_p), ("environment_cubemap_tex", ctypes.c_uint64),
                ("camera", GPUCamera)]


class GPUMaterial(ctypes.Structure):
    _fields_ = [("albedo", ctypes.c_float * 4), ("emissive", ctypes.c_float * 4), ("specular", ctypes.c_float * 4),
                ("roughness", ctypes.c_float), ("specular_percent", ctypes.c_float), ("IOR", ctypes.c_float),
                ("_pad", ctypes.c_float)]


class BuildOptions(ctypes.Structure):
    """rt_build_options (rt_abi.h): exact-preserving speed knobs of the mirror / BVH builders."""
    _fields_ = [("leaf_tree_min", ctypes.c_uint32), ("cut_clusters", ctypes.c_uint32), ("cluster_max", ctypes.c_uint32),
                ("split_angle", ctypes.c_float), ("bvh_small", ctypes.c_uint32), ("host_bvh", ctypes.c_int32),
                ("leaf_screens", ctypes.c_int32)]


class RenderParams(ctypes.Structure):
    _fields_ = [("surface", ctypes.c_void_p), ("surface_last_frame", ctypes.c_void_p),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("pitch", ctypes.c_uint64),
                ("frame_index", ctypes.c_int32), ("spp", ctypes.c_int32), ("bounces", ctypes.c_int32),
                ("shard_index", ctypes.c_int32), ("shard_count", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("out_shard", ctypes.c_void_p), ("stats", ctypes.c_void_p), ("segment_counter", ctypes.c_void_p),
                ("tile_list", ctypes.c_void_p), ("tile_count", ctypes.c_int64), ("wave_clock", ctypes.c_void_p),
                ("tune", ctypes.c_uint32), ("lane_slots", ctypes.c_void_p), ("lane_slot_count", ctypes.c_int64),
                ("lane_cost", ctypes.c_void_p), ("priority_waves", ctypes.c_int64), ("refill_lanes", ctypes.c_int32),
                ("waves_per_simd", ctypes.c_int32), ("lone_slots", ctypes.c_void_p), ("lone_count", ctypes.c_int64)]


assert ctypes.sizeof(GPUScene) == 136 and ctypes.sizeof(GPUMaterial) == 64

# name -> (restype, argtypes); every symbol include/rt_abi.h declares.
_P, _I, _U32, _U64, _F, _SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float, ctypes.c_size_t
_FP = ctypes.POINTER(ctypes.c_float)
SIGNATURES = {
    "raytracing_process": (None, [_P, _P, _I, _I, _SZ, _I, _P]),
    "init_rng": (None, [_U32, _U32, _P, ctypes.c_uint]),
    "rt_render": (_I, [ctypes.POINTER(RenderParams), _P, _P]),
    "rt_foreign_mirror_wait": (_I, [_P]),
    "rt_foreign_last_tracer": (_I, [_P]),
    "rt_experimental_loaded": (_I, []),
    "rt_init_rng": (_I, [_P, _I, _I, _I, _I, _U32, _P]),
    "rt_shard_tiles": (ctypes.c_int64, [_I, _I, _I, _I]),
    "rt_unshard": (_I, [_P, _U64, _I, _I, _I, _P, ctypes.c_int64, _P]),
    "rt_shard_plan_capacity": (ctypes.c_int64, [_I, _I, _I]),
    "rt_shard_plan": (_I, [_I, _I, _I, _P, ctypes.c_int64, _P, _P]),
    "rt_get_build_options": (None, [_P]),
    "rt_set_build_options": (_I, [_P]),
    "rt_lane_plan_capacity": (ctypes.c_int64, [ctypes.c_int64]),
    "rt_lane_plan": (ctypes.c_int64, [_P, ctypes.c_int64, ctypes.c_double, ctypes.c_double, _P, ctypes.c_int64, _P]),
    "rt_lone_plan": (ctypes.c_int64, [_P, ctypes.c_int64, ctypes.c_int64, _U32, _P]),
    "rt_lane_refine": (ctypes.c_int64, [_P, ctypes.c_int64, _P, ctypes.c_int64, _P, ctypes.c_double, _P, ctypes.c_int64,
                                        _P]),
    "rt_init_rng_tiles": (_I, [_P, _I, _I, _P, ctypes.c_int64, _U32, _P]),
    "rt_unshard_tiles": (_I, [_P, _U64, _I, _I, _I, _P, ctypes.c_int64, _P, _P]),
    "rt_comm_unique_id": (_I, [_P]),
    "rt_comm_init_rank": (_I, [ctypes.POINTER(_P), _I, _I, _P]),
    "rt_comm_init_all": (_I, [_P, _I, _P]),
    "rt_comm_destroy": (_I, [_P]),
    "rt_comm_rank": (_I, [_P]),
    "rt_comm_size": (_I, [_P]),
    "rt_comm_group_start": (_I, []),
    "rt_comm_group_end": (_I, []),
    "rt_gather_shards": (_I, [_P, _P, _SZ, _P, _SZ, _P, _I, _P]),
    "rt_tonemap_srgb8": (_I, [_P, _U64, _I, _I, _P, _P]),
    "rt_write_pfm": (_I, [ctypes.c_char_p, _P, _U64, _I, _I]),
    "rt_write_ppm": (_I, [ctypes.c_char_p, _P, _I, _I]),
    "rt_set_device": (_I, [_I]),
    "rt_device_count": (_I, []),
    "rt_malloc": (_I, [ctypes.POINTER(_P), _SZ]),
    "rt_malloc_pitch": (_I, [ctypes.POINTER(_P), ctypes.POINTER(_SZ), _SZ, _SZ]),
    "rt_free": (_I, [_P]),
    "rt_memcpy_h2d": (_I, [_P, _P, _SZ]),
    "rt_memcpy_d2h": (_I, [_P, _P, _SZ]),
    "rt_memcpy_d2d": (_I, [_P, _P, _SZ]),
    "rt_memset": (_I, [_P, _I, _SZ]),
    "rt_synchronize": (_I, []),
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_cubemap_create": (_U64, [_FP, _I]),
    "rt_cubemap_destroy": (_I, [_U64]),
    "rt_scene_create": (_P, []),
    "rt_scene_destroy": (None, [_P]),
    "rt_scene_add_material": (_U32, [_P, ctypes.POINTER(GPUMaterial)]),
    "rt_scene_add_triangle": (None, [_P, _FP, _FP, _FP, _I]),
    "rt_scene_add_quad": (None, [_P, _FP, _FP, _FP, _FP, _I]),
    "rt_scene_add_sphere": (None, [_P, _FP, _F, _I]),
    "rt_scene_add_mesh_file": (_I, [_P, ctypes.c_char_p, _FP, _I]),
    "rt_scene_set_environment_file": (_I, [_P, ctypes.c_char_p]),
    "rt_scene_environment": (_I, [_P, ctypes.POINTER(_P), ctypes.POINTER(_I)]),
    "rt_scene_set_camera": (None, [_P, _FP, _F, _F]),
    "rt_scene_set_viewport": (None, [_P, _I, _I]),
    "rt_scene_upload": (_I, [_P, _P]),
    "rt_scene_gpu": (ctypes.POINTER(GPUScene), [_P]),
    "rt_scene_setup": (_I, [_P, _I, ctypes.c_char_p]),
    "rt_scene_setup_plane": (_I, [_P, _I, ctypes.c_char_p]),
    "rt_scene_build": (None, [_P]),
    "rt_scene_camera": (None, [_P, ctypes.POINTER(GPUCamera)]),
    "rt_scene_host_arrays": (_SZ, [_P, ctypes.POINTER(_P), ctypes.POINTER(_SZ), ctypes.POINTER(_P),
                                   ctypes.POINTER(_SZ), ctypes.POINTER(_P), ctypes.POINTER(_SZ), ctypes.POINTER(_P)]),
    "rt_scene_bvh_max_depth": (_I, [_P]),
    "rt_bvh_build_device": (_I, [_P, _U32, _P, _U32, _P, _P, ctypes.POINTER(_U32), ctypes.POINTER(_I), _P]),
    "rt_scene_mirror_info": (_I, [_P, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
    "rt_scene_mirror_copy": (_I, [_P, _P, _P, _P]),
    "rt_scene_mirror_nodes": (_I, [_P, _P, ctypes.POINTER(_SZ)]),
    "rt_scene_mirror_face_leaf": (_I, [_P, _P, ctypes.POINTER(_SZ)]),
    "rt_scene_mirror_twins": (_I, [_P, _P, ctypes.POINTER(_SZ), _P, ctypes.POINTER(_SZ)]),
    "rt_mirror_build_check": (_I, [_P, _SZ, _P, _SZ, _P, _SZ, _P, _SZ, _P, ctypes.POINTER(ctypes.c_int)]),
    "rt_cluster_cull_host": (_I, [_P, _P, ctypes.c_float, _P]),
    "rt_twin_check_host": (_I, [_P, _P, _P]),
    "rt_xorwow_jump_matrix": (_I, [_I, ctypes.POINTER(ctypes.c_uint32)]),
    "rt_xorwow_init_host": (None, [_U32, _U64, _P]),
}

_lib = None


class RTError(RuntimeError):
    pass


def lib():
    """Load librt_hip.so (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RTError(f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


_exp_lib = None


def load_experimental():
    """Load librt_hip_exp.so: registers the exact alternatives kept for A/B measurement -- the
    wavefront tracer, refill, the lone-pixel kernel and the RT_TUNE A/B kernel variants -- with
    librt_hip.so, whose rt_render refuses them otherwise.  The benchmark's production path never
    needs it."""
    global _exp_lib
    lib()
    if _exp_lib is None:
        if not os.path.exists(EXP_LIB_PATH):
            raise RTError(f"{EXP_LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        _exp_lib = ctypes.CDLL(EXP_LIB_PATH)
    if lib().rt_experimental_loaded() != 1:
        raise RTError("librt_hip_exp.so loaded but its kernels are not registered with librt_hip.so: "
                      + lib().rt_last_error().decode(errors="replace"))
    return _exp_lib


def _check(code, what):
    if code:
        raise RTError(f"{what} failed ({code}): {lib().rt_last_error().decode(errors='replace')}")


def _f3(v):
    return (ctypes.c_float * 3)(*[float(x) for x in v])


def _stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class Scene:
    """RayTracing::Scene mirror (RayTracing/Scene.h:87-129)."""

    def __init__(self):
        self.handle = lib().rt_scene_create()
        if not self.handle:
            raise RTError("rt_scene_create failed")

    def __del__(self):
        if getattr(self, "handle", None) and _lib is not None:
            _lib.rt_scene_destroy(self.handle)
            self.handle = None

    # --- building (Scene.cpp:46-139) -------------------------------------------------
    def add_material(self, albedo=(0, 0, 0), emissive=(0, 0, 0), specular=(0, 0, 0, 0), roughness=0.9,
                     specular_percent=0.0, ior=1.0):
        m = GPUMaterial()
        m.albedo[:] = [*map(float, albedo[:3]), 1.0]
        m.emissive[:] = [*map(float, emissive[:3]), 1.0]
        m.specular[:] = [*map(float, (list(specular) + [0.0])[:4])]
        m.roughness, m.specular_percent, m.IOR = roughness, specular_percent, ior
        return lib().rt_scene_add_material(self.handle, ctypes.byref(m))

    def add_triangle(self, a, b, c, material=0):
        lib().rt_scene_add_triangle(self.handle, _f3(a), _f3(b), _f3(c), material)

    def add_quad(self, a, b, c, d, material=0):
        lib().rt_scene_add_quad(self.handle, _f3(a), _f3(b), _f3(c), _f3(d), material)

    def add_sphere(self, position, radius, material=0):
        lib().rt_scene_add_sphere(self.handle, _f3(position), float(radius), material)

    def add_loaded_scene(self, mesh_path, transform, material=0):
        t = (ctypes.c_float * 16)(*[float(x) for x in transform])
        _check(lib().rt_scene_add_mesh_file(self.handle, mesh_path.encode(), t, material), "add_loaded_scene")

    def set_environment(self, path):
        _check(lib().rt_scene_set_environment_file(self.handle, path.encode()), "set_environment")

    def environment(self):
        """Host copy of the level-0 cube texels [6, size, size, 4] (None when no sky is set)."""
        p, n = ctypes.c_void_p(), ctypes.c_int()
        _check(lib().rt_scene_environment(self.handle, ctypes.byref(p), ctypes.byref(n)), "rt_scene_environment")
        if not p.value:
            return None
        k = n.value
        buf = ctypes.string_at(p.value, 6 * k * k * 16)
        return np.frombuffer(buf, dtype=np.float32).reshape(6, k, k, 4).copy()

    def setup(self, which="bunny", assets_dir=ASSETS_DIR):
        """CUDARayTracer::SetupCornellBox + SetupStanfordBunny (or the config-4/5 scenes)."""
        _check(lib().rt_scene_setup(self.handle, SCENES[which], assets_dir.encode()), f"setup({which})")

    def setup_plane(self, n=708, assets_dir=ASSETS_DIR):
        _check(lib().rt_scene_setup_plane(self.handle, int(n), assets_dir.encode()), f"setup_plane({n})")

    def set_camera(self, position=(0, 0, 0), angle_x=0.0, angle_y=180.0):
        lib().rt_scene_set_camera(self.handle, _f3(position), float(angle_x), float(angle_y))

    def set_viewport(self, width, height):
        lib().rt_scene_set_viewport(self.handle, int(width), int(height))

    def upload(self, rng_state_ptr):
        """Scene::Upload (Scene.cpp:182-234): BVH build if dirty, H2D copies, GPUScene fill."""
        _check(lib().rt_scene_upload(self.handle, ctypes.c_void_p(rng_state_ptr)), "upload")

    @property
    def gpu(self):
        return lib().rt_scene_gpu(self.handle)

    def build(self):
        """Host half of upload (camera + BVH) with no device work."""
        lib().rt_scene_build(self.handle)

    def camera(self):
        c = GPUCamera()
        lib().rt_scene_camera(self.handle, ctypes.byref(c))
        return c

    def max_depth(self):
        return lib().rt_scene_bvh_max_depth(self.handle)

    def mirror(self, trees=False):
        """The kernel's triangle mirror built on the host (mirror.h): leaf-ordered (N,12) float32
        records (v0, e1, e2, face id bits, pair/tree index, flag); with trees=True also the leaf
        trees: nodes (K,16) and their triangle records (M,12) (leaftree.h)."""
        import numpy as np
        n = [ctypes.c_size_t() for _ in range(3)]
        _check(lib().rt_scene_mirror_info(self.handle, *[ctypes.byref(x) for x in n]), "rt_scene_mirror_info")
        tris = np.zeros((n[0].value, 12), dtype=np.float32)
        tree = np.zeros((n[1].value, 16), dtype=np.float32)
        ltris = np.zeros((n[2].value, 12), dtype=np.float32)
        _check(lib().rt_scene_mirror_copy(self.handle, tris.ctypes.data, tree.ctypes.data, ltris.ctypes.data),
               "rt_scene_mirror_copy")
        return (tris, tree, ltris) if trees else tris

    def mirror_nodes(self):
        """The traversal's private node array (mirror.h nodes) as (N, 8) float32 (uint32 view for
        first / count)."""
        import numpy as np
        n = ctypes.c_size_t()
        _check(lib().rt_scene_mirror_nodes(self.handle, None, ctypes.byref(n)), "rt_scene_mirror_nodes")
        out = np.zeros((n.value, 8), dtype=np.float32)
        _check(lib().rt_scene_mirror_nodes(self.handle, out.ctypes.data, ctypes.byref(n)), "rt_scene_mirror_nodes")
        return out

    def mirror_face_leaf(self):
        """Scenes with big leaves: each face's leaf in the private node array (uint32; 0xffffffff none,
        0xfffffffe two leaves), the deferred leaves' guard table (rt_fast.h); empty otherwise."""
        import numpy as np
        n = ctypes.c_size_t()
        _check(lib().rt_scene_mirror_face_leaf(self.handle, None, ctypes.byref(n)), "rt_scene_mirror_face_leaf")
        out = np.zeros(n.value, dtype=np.uint32)
        if n.value:
            _check(lib().rt_scene_mirror_face_leaf(self.handle, out.ctypes.data, ctypes.byref(n)), "rt_scene_mirror_face_leaf")
        return out

    def mirror_twins(self):
        """The big leaves' twin records (mirror.h): quads (Q, 28) and units (U, 16) float32."""
        import numpy as np
        nq, nu = ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib().rt_scene_mirror_twins(self.handle, None, ctypes.byref(nq), None, ctypes.byref(nu)), "rt_scene_mirror_twins")
        q = np.zeros((nq.value, 28), dtype=np.float32)
        u = np.zeros((nu.value, 16), dtype=np.float32)
        _check(lib().rt_scene_mirror_twins(self.handle, q.ctypes.data, ctypes.byref(nq), u.ctypes.data, ctypes.byref(nu)),
               "rt_scene_mirror_twins")
        return q, u

    def host_arrays(self):
        """numpy copies of the host arrays: nodes (N,8) f32/u32 view, face indices, vertices, faces."""
        import numpy as np
        ptrs = [ctypes.c_void_p() for _ in range(4)]
        counts = [ctypes.c_size_t() for _ in range(3)]
        lib().rt_scene_host_arrays(self.handle, ctypes.byref(ptrs[0]), ctypes.byref(counts[0]), ctypes.byref(ptrs[1]),
                                   ctypes.byref(counts[1]), ctypes.byref(ptrs[2]), ctypes.byref(counts[2]),
                                   ctypes.byref(ptrs[3]))

        def grab(p, nbytes):
            if not p.value or nbytes == 0:
                return np.zeros(0, dtype=np.uint8)
            return np.frombuffer(ctypes.string_at(p.value, nbytes), dtype=np.uint8).copy()

        nn, nf, nv = counts[0].value, counts[1].value, counts[2].value
        return {"nodes": grab(ptrs[0], nn * 32), "face_indices": grab(ptrs[1], nf * 4),
                "vertices": grab(ptrs[2], nv * 32), "faces": grab(ptrs[3], nf * 16)}


def mirror_build_check(nodes, face_indices, faces, vertices):
    """rt_mirror_build_check: the host mirror of raw reference arrays (numpy: nodes (N,8) 32-bit, face
    indices u32, faces (F,4) u32, vertices (V,8) f32) -> (words 10-11 of every record as (n, 2) uint32,
    whether twin records were built)."""
    import numpy as np
    nodes, fi = np.ascontiguousarray(nodes), np.ascontiguousarray(face_indices, dtype=np.uint32)
    faces, vertices = np.ascontiguousarray(faces), np.ascontiguousarray(vertices)
    meta = np.zeros((fi.size, 2), dtype=np.uint32)
    tw = ctypes.c_int(0)
    _check(lib().rt_mirror_build_check(nodes.ctypes.data, nodes.shape[0], fi.ctypes.data, fi.size, faces.ctypes.data,
                                       faces.shape[0], vertices.ctypes.data, vertices.shape[0], meta.ctypes.data,
                                       ctypes.byref(tw)), "rt_mirror_build_check")
    return meta, bool(tw.value)


def bvh_build_device(vertices, faces, stream=None):
    """BVH::Calculate on the GPU (rt_bvh_build_device) from device tensors of GPUVertex (N,8) f32
    and GPUFace (F,4) u32 rows; returns (nodes (2F-1, 8) f32 device tensor, face_indices (F,) int32
    device tensor, node_count, max_depth)."""
    import torch
    nf = faces.shape[0]
    nodes = torch.empty((max(1, 2 * nf - 1), 8), dtype=torch.float32, device=faces.device)
    fi = torch.empty((nf,), dtype=torch.int32, device=faces.device)
    count, depth = _U32(0), _I(0)
    _check(lib().rt_bvh_build_device(vertices.data_ptr(), vertices.shape[0], faces.data_ptr(), nf, nodes.data_ptr(),
                                     fi.data_ptr(), ctypes.byref(count), ctypes.byref(depth), _stream_ptr(stream)),
           "rt_bvh_build_device")
    return nodes, fi, count.value, depth.value


def alloc_surface(width, height, device=None):
    """A pitched float4 surface (RGBA fp32), rows padded to a 256-byte pitch like cudaMallocPitch."""
    row_floats = ((width * 16 + 255) // 256) * 256 // 4
    t = torch.zeros((height, row_floats), dtype=torch.float32, device=device or "cuda")
    return t


def surface_view(t, width):
    """[H, W, 4] view of a pitched surface tensor."""
    return t[:, : width * 4].reshape(t.shape[0], width, 4)


def alloc_rng(count, device=None):
    return torch.zeros((count * RNG_STATE_BYTES // 4,), dtype=torch.int32, device=device or "cuda")


def init_rng_states(rng, width, height, seed, shard_index=0, shard_count=1, stream=None):
    _check(lib().rt_init_rng(ctypes.c_void_p(rng.data_ptr()), width, height, shard_index, shard_count, seed,
                             _stream_ptr(stream)), "rt_init_rng")


def render(scene, surface, last, width, height, spp, bounces, frame_index=0, shard_index=0, shard_count=1,
           out_shard=None, stats=None, segment_counter=None, stream=None, tracer="fast", tile_list=None,
           wave_clock=None, tune=0, lane_slots=None, lane_cost=None, priority_waves=0, refill_lanes=0,
           waves_per_simd=0, lone_slots=None, validate=False):
    """rt_render: one frame (or one shard of it) on `stream` (default: torch's current stream).
    tile_list: device int32 tensor of tile ids (a row of a sharding.Plan) instead of the
    round-robin deal; wave_clock: device int64 tensor [entries*4] receiving per-wave clocks;
    tune: diagnostic A/B knobs (0 = production); lane_slots: device int32 lane map (rt_lane_plan,
    a multiple of 64 entries); lane_cost: device int32/uint32 [slots] receiving per-pixel work;
    lone_slots: device int32 slots for the lone-pixel kernel (rt_lone_plan; needs lane_slots);
    validate: RT_RENDER_VALIDATE (lone_slots and lane_slots checked disjoint first; synchronises)."""
    p = RenderParams()
    if lone_slots is not None and lone_slots.numel() > 0:
        assert lone_slots.dtype == torch.int32 and lone_slots.is_cuda and lone_slots.dim() == 1
        p.lone_slots, p.lone_count = lone_slots.data_ptr(), lone_slots.numel()
    if lane_slots is not None:
        assert lane_slots.dtype == torch.int32 and lane_slots.is_cuda and lane_slots.numel() % 64 == 0
        p.lane_slots, p.lane_slot_count = lane_slots.data_ptr(), lane_slots.numel()
        p.priority_waves = int(priority_waves)
    if lane_cost is not None:
        assert lane_cost.dtype == torch.int32 and lane_cost.is_cuda
        p.lane_cost = lane_cost.data_ptr()
    if tile_list is not None:
        assert tile_list.dtype == torch.int32 and tile_list.is_cuda and tile_list.dim() == 1
        p.tile_list, p.tile_count = tile_list.data_ptr(), tile_list.numel()
    if wave_clock is not None:
        n = tile_list.numel() if tile_list is not None else tiles_of(width, height, shard_index, shard_count)
        waves = lane_slots.numel() // 64 if lane_slots is not None else 4 * n
        assert wave_clock.dtype == torch.int64 and wave_clock.numel() >= waves
        p.wave_clock = wave_clock.data_ptr()
    p.tune = int(tune)
    p.refill_lanes = int(refill_lanes)
    p.waves_per_simd = int(waves_per_simd)
    p.surface = surface.data_ptr() if surface is not None else None
    p.surface_last_frame = last.data_ptr() if last is not None else None
    p.width, p.height = width, height
    p.pitch = surface.shape[1] * 4 if surface is not None else width * 16
    p.frame_index, p.spp, p.bounces = frame_index, spp, bounces
    p.shard_index, p.shard_count = shard_index, shard_count
    p.out_shard = out_shard.data_ptr() if out_shard is not None else None
    p.flags = TRACERS[tracer] | (RT_RENDER_VALIDATE if validate else 0)
    if segment_counter is not None:
        p.segment_counter = segment_counter.data_ptr()
    if stats is not None:
        p.flags |= RT_RENDER_STATS
        p.stats = stats.data_ptr()
    gpu = scene.gpu if hasattr(scene, "gpu") else ctypes.pointer(scene)  # Scene, or a GPUScene filled by the caller
    _check(lib().rt_render(ctypes.byref(p), ctypes.cast(gpu, ctypes.c_void_p), _stream_ptr(stream)), "rt_render")


def foreign_mirror_wait(gpu_scene):
    """rt_foreign_mirror_wait: block until the background mirror build of a foreign GPUScene (a
    ctypes GPUScene filled by the caller) has finished; the next render installs it."""
    _check(lib().rt_foreign_mirror_wait(ctypes.byref(gpu_scene)), "rt_foreign_mirror_wait")


def foreign_last_tracer(gpu_scene):
    """rt_foreign_last_tracer: 1 production tracer, 0 reference layout (fingerprint mismatch),
    -1 no mirror yet (test diagnostics; synchronises the device)."""
    return int(lib().rt_foreign_last_tracer(ctypes.byref(gpu_scene)))


def cluster_cull_host(origin, nd, best, node):
    """The render kernel's leaf-tree cull predicate (rt_fast.h cluster_cull) on the host."""
    import numpy as np
    o = np.ascontiguousarray(origin, dtype=np.float32)
    d = np.ascontiguousarray(nd, dtype=np.float32)
    k = np.ascontiguousarray(node, dtype=np.float32)
    return bool(lib().rt_cluster_cull_host(o.ctypes.data, d.ctypes.data, float(best), k.ctypes.data))


def shard_tiles(width, height, shard_index, shard_count):
    return int(lib().rt_shard_tiles(width, height, shard_index, shard_count))


tiles_of = shard_tiles


def shard_plan(width, height, shard_count, tile_cost=None):
    """rt_shard_plan: (tile_lists int32 [shard_count, capacity] -1 padded, counts int64 [shard_count])
    on the host; tile_cost None = round-robin, else longest-processing-time-first."""
    cap = int(lib().rt_shard_plan_capacity(width, height, shard_count))
    lists = np.zeros((shard_count, cap), dtype=np.int32)
    counts = np.zeros((shard_count,), dtype=np.int64)
    cost_ptr = None
    if tile_cost is not None:
        cost = np.ascontiguousarray(tile_cost, dtype=np.float64)
        assert cost.size == sharding.tiles_total(width, height)
        cost_ptr = cost.ctypes.data
    _check(lib().rt_shard_plan(width, height, shard_count, cost_ptr, cap, lists.ctypes.data, counts.ctypes.data),
           "rt_shard_plan")
    return lists, counts


def build_options():
    """Current rt_build_options (a BuildOptions)."""
    o = BuildOptions()
    lib().rt_get_build_options(ctypes.byref(o))
    return o


def set_build_options(**changes):
    """rt_set_build_options with the given fields changed (no arguments: the defaults)."""
    if not changes:
        _check(lib().rt_set_build_options(None), "rt_set_build_options")
        return
    o = build_options()
    for k, v in changes.items():
        setattr(o, k, v)
    _check(lib().rt_set_build_options(ctypes.byref(o)), "rt_set_build_options")


def lane_plan(cost, parallel_units=48000.0, slack=1.0):
    """rt_lane_plan: (int32 numpy lane map, number of leading long waves) from per-slot work
    (numpy uint32/int32 [slots], a probe frame's lane_cost)."""
    cost = np.ascontiguousarray(np.asarray(cost).astype(np.uint32))
    cap = int(lib().rt_lane_plan_capacity(cost.size))
    out = np.empty(max(cap, 1), dtype=np.int32)
    nlong = ctypes.c_int64(0)
    n = int(lib().rt_lane_plan(cost.ctypes.data, cost.size, float(parallel_units), float(slack), out.ctypes.data, cap,
                               ctypes.byref(nlong)))
    if n < 0:
        raise RTError("rt_lane_plan failed: " + lib().rt_last_error().decode(errors="replace"))
    return out[:n].copy(), int(nlong.value)


def lane_refine(lane_map, cost, wave_ticks, theta=0.75):
    """rt_lane_refine: (int32 numpy lane map, waves made by splitting) -- the waves of `lane_map`
    whose measured clock (numpy int64 [waves], a timing frame's wave_clock) is within theta of the
    longest split in two, all waves ordered longest first."""
    m = np.ascontiguousarray(np.asarray(lane_map, dtype=np.int32).ravel())
    cost = np.ascontiguousarray(np.asarray(cost).astype(np.uint32))
    ticks = np.ascontiguousarray(np.asarray(wave_ticks, dtype=np.int64))
    assert m.size % 64 == 0 and ticks.size >= m.size // 64
    out = np.empty(2 * m.size, dtype=np.int32)
    nsplit = ctypes.c_int64(0)
    n = int(lib().rt_lane_refine(m.ctypes.data, m.size, cost.ctypes.data, cost.size, ticks.ctypes.data, float(theta),
                                 out.ctypes.data, out.size, ctypes.byref(nsplit)))
    if n < 0:
        raise RTError("rt_lane_refine failed: " + lib().rt_last_error().decode(errors="replace"))
    return out[:n].copy(), int(nsplit.value)


def lone_plan(cost, max_lone, min_cost=1):
    """rt_lone_plan: (int32 numpy lone slots, heaviest first; the cost array with those slots marked
    for rt_lane_plan) from per-slot work (a probe frame's lane_cost)."""
    cost = np.ascontiguousarray(np.asarray(cost).astype(np.uint32)).copy()
    out = np.empty(max(int(max_lone), 1), dtype=np.int32)
    n = int(lib().rt_lone_plan(cost.ctypes.data, cost.size, int(max_lone), int(min_cost), out.ctypes.data))
    if n < 0:
        raise RTError("rt_lone_plan failed: " + lib().rt_last_error().decode(errors="replace"))
    return out[:n].copy(), cost


def init_rng_tiles(rng, width, height, tile_list, seed, stream=None):
    """rt_init_rng_tiles: compact states for a device int32 tile list."""
    _check(lib().rt_init_rng_tiles(ctypes.c_void_p(rng.data_ptr()), width, height, ctypes.c_void_p(tile_list.data_ptr()),
                                   tile_list.numel(), seed, _stream_ptr(stream)), "rt_init_rng_tiles")


def unshard_tiles(surface, width, height, shards, tile_lists, stream=None):
    """rt_unshard_tiles: shards [N, capacity*256, 4] f32, tile_lists device int32 [N, capacity]."""
    n, cap = tile_lists.shape
    _check(lib().rt_unshard_tiles(ctypes.c_void_p(surface.data_ptr()), surface.shape[1] * 4, width, height, n,
                                  ctypes.c_void_p(shards.data_ptr()), cap, ctypes.c_void_p(tile_lists.data_ptr()),
                                  _stream_ptr(stream)), "rt_unshard_tiles")


class Comm:
    """rt_comm (RCCL) for the frame-end gather.  Rank 0 makes the id (``unique_id()``); the caller
    hands it to every rank; each rank constructs ``Comm(nranks, rank, id)`` on its device."""

    ID_BYTES = 128

    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * Comm.ID_BYTES)()
        _check(lib().rt_comm_unique_id(buf), "rt_comm_unique_id")
        return bytes(buf)

    def __init__(self, nranks, rank, uid):
        assert len(uid) == Comm.ID_BYTES
        self.handle = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * Comm.ID_BYTES)(*uid)
        _check(lib().rt_comm_init_rank(ctypes.byref(self.handle), nranks, rank, buf), "rt_comm_init_rank")
        self.rank, self.nranks = rank, nranks

    def gather(self, shard, shard_bytes, gathered=None, stride=0, recv_bytes=None, root=0, stream=None):
        rb = None
        if recv_bytes is not None:
            rb = (ctypes.c_size_t * self.nranks)(*[int(b) for b in recv_bytes])
        _check(lib().rt_gather_shards(self.handle, ctypes.c_void_p(shard.data_ptr()), int(shard_bytes),
                                      ctypes.c_void_p(gathered.data_ptr() if gathered is not None else None),
                                      int(stride), rb, root, _stream_ptr(stream)), "rt_gather_shards")

    def close(self):
        if self.handle:
            _check(lib().rt_comm_destroy(self.handle), "rt_comm_destroy")
            self.handle = ctypes.c_void_p()


def unshard(surface, width, height, shard_count, shards, per_shard, stream=None):
    _check(lib().rt_unshard(ctypes.c_void_p(surface.data_ptr()), surface.shape[1] * 4, width, height, shard_count,
                            ctypes.c_void_p(shards.data_ptr()), per_shard, _stream_ptr(stream)), "rt_unshard")


def tonemap(surface, width, height, stream=None):
    """The reference viewer's display transform (main.cpp:78-94 into an sRGB back buffer):
    [H, W, 3] uint8 on the GPU, rows top to bottom."""
    out = torch.empty((height, width, 3), dtype=torch.uint8, device=surface.device)
    _check(lib().rt_tonemap_srgb8(ctypes.c_void_p(surface.data_ptr()), surface.shape[1] * 4, width, height,
                                  ctypes.c_void_p(out.data_ptr()), _stream_ptr(stream)), "rt_tonemap_srgb8")
    return out


def write_pfm(path, surface, width, height):
    """Linear RGB of a pitched float4 surface (torch, any device; or a numpy [H, row] array) as
    PFM, rows bottom to top -- the surface's own order."""
    host = surface.detach().to("cpu").contiguous().numpy() if isinstance(surface, torch.Tensor) else np.ascontiguousarray(surface, dtype=np.float32)
    _check(lib().rt_write_pfm(os.fsencode(path), host.ctypes.data, host.shape[1] * 4, width, height), "rt_write_pfm")


def write_ppm(path, rgb):
    """[H, W, 3] uint8 (tonemap's output, any device) as binary PPM."""
    host = rgb.detach().to("cpu").contiguous().numpy() if isinstance(rgb, torch.Tensor) else np.ascontiguousarray(rgb, dtype=np.uint8)
    _check(lib().rt_write_ppm(os.fsencode(path), host.ctypes.data, host.shape[1], host.shape[0]), "rt_write_ppm")


def raytracing_process(surface, last, width, height, frame_index, scene):
    """The reference entry point (main_raytracing.cu:202): spp 5, 6 bounces, null stream."""
    lib().raytracing_process(ctypes.c_void_p(surface.data_ptr()), ctypes.c_void_p(last.data_ptr()), width, height,
                             surface.shape[1] * 4, frame_index, ctypes.cast(scene.gpu, ctypes.c_void_p))


def init_rng(thread_block_count, thread_block_size, rng, seed):
    """The reference entry point (Random.cu:10)."""
    lib().init_rng(thread_block_count, thread_block_size, ctypes.c_void_p(rng.data_ptr()), seed)


class RayTracer:
    """CUDARayTracer mirror (RayTracing/RayTracing.{h,cpp}), headless.

    ``process()`` = one progressive frame: lazy RNG init (fixed seed instead of the
    reference's time-based one), camera update + upload, render, copy to the last-frame
    surface, frame_index++ (RayTracing.cpp:205-234).
    """

    def __init__(self, width, height, scene="bunny", spp=REFERENCE_SPP, bounces=REFERENCE_BOUNCES, seed=0xDEADBEEF):
        self.width, self.height, self.spp, self.bounces, self.seed = width, height, spp, bounces, seed
        self.scene = Scene()
        self.scene.setup(scene)
        self.surface = alloc_surface(width, height)
        self.last_frame = alloc_surface(width, height)
        self.rng = None
        self.frame_index = 0

    def on_resize(self, width, height):
        self.width, self.height = width, height
        self.surface = alloc_surface(width, height)
        self.last_frame = alloc_surface(width, height)
        self.rng = None
        self.frame_index = 0

    def process(self, stats=None):
        if self.rng is None:
            self.rng = alloc_rng(self.width * self.height)
            init_rng_states(self.rng, self.width, self.height, self.seed)
        self.scene.set_viewport(self.width, self.height)
        self.scene.upload(self.rng.data_ptr())
        render(self.scene, self.surface, self.last_frame, self.width, self.height, self.spp, self.bounces,
               frame_index=self.frame_index, stats=stats)
        self.last_frame.copy_(self.surface)
        self.frame_index += 1
        return surface_view(self.surface, self.width)

    def save(self, path):
        """The current frame: ``.pfm`` linear RGB, ``.ppm`` as the reference's viewer shows it
        (exposure 0.5, ACES film, sRGB; main.cpp:78-94, 438)."""
        if str(path).lower().endswith(".pfm"):
            write_pfm(path, self.surface, self.width, self.height)
        elif str(path).lower().endswith(".ppm"):
            write_ppm(path, tonemap(self.surface, self.width, self.height))
        else:
            raise ValueError("RayTracer.save: .pfm or .ppm")


from . import sharding  # noqa: E402  (multi-GPU tile bookkeeping; the data path is in librt_hip.so)

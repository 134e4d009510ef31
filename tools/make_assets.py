"""Convert the reference's input data files into the binary assets this repo ships.

Run in the survey container only (it reads /root/reference, which does not exist on the
GPU box).  Outputs, both committed under assets/:

* assets/bunny_mesh.bin  -- the Stanford bunny exactly as the reference's importer hands it
  to Scene::AddLoadedScene (RayTracing/Scene.cpp:75-132): the mesh returned by assimp with
  aiProcess_Triangulate | JoinIdenticalVertices | GenSmoothNormals | SortByPType and
  AI_CONFIG_PP_GSN_MAX_SMOOTHING_ANGLE = 100 (utils/AssimpLoader.cpp:29-51).  The
  reference pins assimp through vcpkg without a version (vcpkg.json:4-7); the importer
  used here is the assimp 3.3 that is statically linked into
  /opt/conda/plugins/sceneparsers/libassimpsceneimport.so (C API via ctypes).  The
  bunny's OBJ node transform is identity, so the node transform is not stored; the
  -90 degree X rotation the reference applies at the root (AssimpLoader.cpp:47-48) is
  applied by the C++ loader, exactly as CopyNodes does.
  Layout: magic 'RTMESH01', u32 nverts, u32 nfaces, f32[nverts][3] positions,
  f32[nverts][3] normals, u32[nfaces][3] indices.

* assets/sunset_cube128.bin -- level 0 of the six faces of data/sunset_uncompressed.dds
  (legacy DDS, D3DFMT 116 = fp32 RGBA, 128x128, 8 mips, all faces; parsed the way
  utils/image/DDSLoader.cpp:135-371 and utils/CUDATexture.cpp:187-220 slice it: faces are
  stored face-major with all mips of a face contiguous, face order +X,-X,+Y,-Y,+Z,-Z).
  Layout: magic 'RTCUBE01', u32 size, f32[6][size][size][4].
"""
import ctypes
import os
import struct
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "assets")
ASSIMP = "/opt/conda/plugins/sceneparsers/libassimpsceneimport.so"


class aiVector3D(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float)]


class aiFace(ctypes.Structure):
    _fields_ = [("mNumIndices", ctypes.c_uint), ("mIndices", ctypes.POINTER(ctypes.c_uint))]


class aiMesh(ctypes.Structure):  # assimp 3.3 layout (include/assimp/mesh.h)
    _fields_ = [
        ("mPrimitiveTypes", ctypes.c_uint),
        ("mNumVertices", ctypes.c_uint),
        ("mNumFaces", ctypes.c_uint),
        ("mVertices", ctypes.POINTER(aiVector3D)),
        ("mNormals", ctypes.POINTER(aiVector3D)),
        ("mTangents", ctypes.c_void_p),
        ("mBitangents", ctypes.c_void_p),
        ("mColors", ctypes.c_void_p * 8),
        ("mTextureCoords", ctypes.c_void_p * 8),
        ("mNumUVComponents", ctypes.c_uint * 8),
        ("mFaces", ctypes.POINTER(aiFace)),
    ]


class aiNode(ctypes.Structure):
    pass


aiNode._fields_ = [
    ("mName_length", ctypes.c_size_t),
    ("mName_data", ctypes.c_char * 1024),
    ("mTransformation", ctypes.c_float * 16),
    ("mParent", ctypes.POINTER(aiNode)),
    ("mNumChildren", ctypes.c_uint),
    ("mChildren", ctypes.POINTER(ctypes.POINTER(aiNode))),
    ("mNumMeshes", ctypes.c_uint),
    ("mMeshes", ctypes.POINTER(ctypes.c_uint)),
]


class aiScene(ctypes.Structure):
    _fields_ = [
        ("mFlags", ctypes.c_uint),
        ("mRootNode", ctypes.POINTER(aiNode)),
        ("mNumMeshes", ctypes.c_uint),
        ("mMeshes", ctypes.POINTER(ctypes.POINTER(aiMesh))),
    ]


def make_bunny():
    lib = ctypes.CDLL(ASSIMP)
    lib.aiCreatePropertyStore.restype = ctypes.c_void_p
    lib.aiSetImportPropertyFloat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_float]
    lib.aiImportFileExWithProperties.restype = ctypes.POINTER(aiScene)
    lib.aiImportFileExWithProperties.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    lib.aiReleaseImport.argtypes = [ctypes.POINTER(aiScene)]
    store = lib.aiCreatePropertyStore()
    lib.aiSetImportPropertyFloat(store, b"PP_GSN_MAX_SMOOTHING_ANGLE", 100.0)
    flags = 0x8 | 0x2 | 0x40 | 0x8000  # Triangulate | JoinIdenticalVertices | GenSmoothNormals | SortByPType
    sc = lib.aiImportFileExWithProperties(os.path.join(REF, "data/stanford-bunny.obj").encode(), flags, None, store)
    assert sc, "assimp import failed"
    s = sc.contents
    # walk the node tree the way CopyNodes does (AssimpLoader.cpp:8-27); the bunny has one
    # mesh under identity node transforms.
    meshes = []

    def walk(node, depth=0):
        n = node.contents
        t = np.array(n.mTransformation[:], dtype=np.float32)
        assert np.array_equal(t, np.eye(4, dtype=np.float32).ravel()), "non-identity node transform"
        for i in range(n.mNumMeshes):
            meshes.append(n.mMeshes[i])
        for i in range(n.mNumChildren):
            walk(n.mChildren[i], depth + 1)

    walk(s.mRootNode)
    assert meshes == [0], meshes
    m = s.mMeshes[0].contents
    nv, nf = m.mNumVertices, m.mNumFaces
    pos = np.ctypeslib.as_array(ctypes.cast(m.mVertices, ctypes.POINTER(ctypes.c_float)), shape=(nv * 3,)).copy()
    nrm = np.ctypeslib.as_array(ctypes.cast(m.mNormals, ctypes.POINTER(ctypes.c_float)), shape=(nv * 3,)).copy()
    idx = np.empty((nf, 3), dtype=np.uint32)
    for f in range(nf):
        face = m.mFaces[f]
        assert face.mNumIndices == 3
        idx[f] = face.mIndices[0], face.mIndices[1], face.mIndices[2]
    lib.aiReleaseImport(sc)
    with open(os.path.join(OUT, "bunny_mesh.bin"), "wb") as fh:
        fh.write(b"RTMESH01" + struct.pack("<II", nv, nf))
        fh.write(pos.astype("<f4").tobytes())
        fh.write(nrm.astype("<f4").tobytes())
        fh.write(idx.astype("<u4").tobytes())
    print("bunny", nv, nf)


def make_sky():
    b = open(os.path.join(REF, "data/sunset_uncompressed.dds"), "rb").read()
    assert b[:4] == b"DDS "
    hdr = struct.unpack("<31I", b[4:128])
    size, height, width, mips = hdr[0], hdr[2], hdr[3], hdr[6]
    pf_flags, fourcc, caps2 = hdr[19], hdr[20], hdr[27]
    assert size == 124 and width == height and pf_flags & 4 and fourcc == 116
    assert caps2 & 0xFE00 == 0xFE00, "not a full cubemap"
    face_bytes = sum(16 * (width >> m) * (height >> m) for m in range(mips))
    level0 = 16 * width * height
    faces = []
    for f in range(6):
        off = 128 + f * face_bytes
        faces.append(np.frombuffer(b, dtype="<f4", count=level0 // 4, offset=off))
    assert 128 + 6 * face_bytes == len(b)
    with open(os.path.join(OUT, "sunset_cube128.bin"), "wb") as fh:
        fh.write(b"RTCUBE01" + struct.pack("<I", width))
        for f in faces:
            fh.write(f.tobytes())
    print("sky", width, mips)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    make_sky()
    make_bunny()

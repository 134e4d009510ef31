"""Frame output (the viewer path, main.cpp:66-94 + the sRGB back buffer at main.cpp:438):
PFM / PPM writers through the C-ABI (CPU), and the tonemap kernel against a numpy restatement
(GPU).  The tonemap is for viewing: its check is +-1 LSB against fp64 arithmetic."""
import numpy as np
import pytest
import torch

import rt_testlib as T


def _read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline() == b"PF\n"
        w, h = map(int, f.readline().split())
        assert float(f.readline()) == -1.0
        data = np.frombuffer(f.read(), dtype="<f4")
    return data.reshape(h, w, 3)


def _surface(rng, w, h):
    row = ((w * 16 + 255) // 256) * 256 // 4  # rt.alloc_surface's pitch
    s = np.zeros((h, row), dtype=np.float32)
    s[:, : w * 4] = rng.uniform(0, 4, size=(h, w * 4)).astype(np.float32)
    return s


def test_pfm_roundtrip(tmp_path):
    rt = T.load_rt()
    w, h = 37, 11
    s = _surface(np.random.default_rng(1), w, h)
    p = tmp_path / "f.pfm"
    rt.write_pfm(str(p), s, w, h)
    img = _read_pfm(p)
    # rows bottom to top in PFM = the surface's own row order (row 0 = bottom scanline)
    assert np.array_equal(img, s[:, : w * 4].reshape(h, w, 4)[..., :3])


def test_ppm_roundtrip_and_errors(tmp_path):
    rt = T.load_rt()
    rgb = np.random.default_rng(2).integers(0, 256, size=(5, 7, 3), dtype=np.uint8)
    p = tmp_path / "f.ppm"
    rt.write_ppm(str(p), rgb)
    raw = p.read_bytes()
    assert raw.startswith(b"P6\n7 5\n255\n") and raw[len(b"P6\n7 5\n255\n"):] == rgb.tobytes()
    with pytest.raises(rt.RTError, match="cannot open"):
        rt.write_ppm(str(tmp_path / "no" / "such" / "dir.ppm"), rgb)


def _tonemap_ref(rgb):
    x = rgb.astype(np.float64) * 0.5
    with np.errstate(invalid="ignore"):
        y = (x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14)
    y = np.clip(np.nan_to_num(y, nan=0.0), 0, 1)
    s = np.where(y <= 0.0031308, 12.92 * y, 1.055 * np.power(y, 1 / 2.4) - 0.055)
    return np.floor(np.clip(s, 0, 1) * 255 + 0.5).astype(np.int64)


@pytest.mark.gpu
def test_tonemap_matches_numpy():
    rt = T.load_rt()
    w, h = 301, 17
    s = _surface(np.random.default_rng(3), w, h)
    s[3, 8:12] = np.nan  # pixel (2, 3): NaN -> black, as saturate does
    surf = torch.from_numpy(s).cuda()
    got = rt.tonemap(surf, w, h).cpu().numpy().astype(np.int64)
    want = _tonemap_ref(s[:, : w * 4].reshape(h, w, 4)[..., :3])[::-1]  # display rows: top first
    assert np.abs(got - want).max() <= 1
    assert (got[h - 1 - 3, 2] == 0).all()


@pytest.mark.gpu
def test_raytracer_save(tmp_path):
    rt = T.load_rt()
    tr = rt.RayTracer(64, 36, spp=2)
    frame = tr.process().cpu().numpy()
    tr.save(str(tmp_path / "f.pfm"))
    tr.save(str(tmp_path / "f.ppm"))
    assert np.array_equal(_read_pfm(tmp_path / "f.pfm"), frame[..., :3])
    raw = (tmp_path / "f.ppm").read_bytes()
    assert raw.startswith(b"P6\n64 36\n255\n") and len(raw) == len(b"P6\n64 36\n255\n") + 64 * 36 * 3

"""Leaf trees beyond the default threshold: the cooperative tree walk (rt_fast.h coop_tree) with
several tree leaves per scene and on the 345-triangle floor leaf of config 2, against the CPU
oracle bit for bit.  The threshold is lowered through rt_set_build_options (process-wide; the
mirror is built at upload) and restored afterwards.
"""
import numpy as np
import pytest
import torch

import rt_testlib as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case,tree_min", [(("bunny", 96, 54, 4, 6), 300), (("bunny4", 64, 36, 2, 6), 200)])
def test_coop_tree_more_leaves(case, tree_min):
    rt = T.load_rt()
    torch.cuda.set_device(0)
    which, w, h, spp, bounces = case
    rt.set_build_options(leaf_tree_min=tree_min)
    try:
        s = rt.Scene()
        s.setup(which)
        s.set_viewport(w, h)
        rng = rt.alloc_rng(w * h)
        rt.init_rng_states(rng, w, h, T.SEED)
        s.upload(rng.data_ptr())
        _, tree, _ = s.mirror(trees=True)
        a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
        rt.render(s, a, b, w, h, spp, bounces)
        torch.cuda.synchronize()
    finally:
        rt.set_build_options()
    assert len(tree) > 0, "the lowered threshold did not produce leaf trees"
    got = rt.surface_view(a, w).cpu().numpy()
    want = T.OracleScene(which).render(w, h, spp, bounces)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), float(np.nanmax(np.abs(got - want)))


def test_build_options_validated():
    rt = T.load_rt()
    d = rt.build_options()
    assert (d.leaf_tree_min, d.cut_clusters, d.cluster_max, d.bvh_small, d.host_bvh) == (1024, 32, 16, 16, 0)
    with pytest.raises(rt.RTError, match="build_options"):
        rt.set_build_options(cluster_max=99)
    assert rt.build_options().cluster_max == 16

"""Leaf trees beyond the default threshold: the cooperative tree walk (rt_fast.h coop_tree) with
several tree leaves per scene and on the 345-triangle floor leaf of config 2, against the CPU
oracle bit for bit.  The mirror reads RT_LEAF_TREE_MIN once per process, so each case renders in
a child process with the threshold lowered (one GPU process at a time).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import rt_testlib as T

pytestmark = pytest.mark.gpu

CHILD = r"""
import json, sys
import numpy as np, torch
sys.path.insert(0, {tests!r}); sys.path.insert(0, {root!r})
import rt_testlib as T
rt = T.load_rt()
torch.cuda.set_device(0)
which, w, h, spp, bounces = {case!r}
s = rt.Scene(); s.setup(which); s.set_viewport(w, h)
rng = rt.alloc_rng(w * h); rt.init_rng_states(rng, w, h, T.SEED); s.upload(rng.data_ptr())
_, tree, _ = s.mirror(trees=True)
a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
rt.render(s, a, b, w, h, spp, bounces)
got = rt.surface_view(a, w).cpu().numpy()
want = T.OracleScene(which).render(w, h, spp, bounces)
print(json.dumps({{"tree_nodes": int(len(tree)), "same": bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))),
                  "maxdiff": float(np.nanmax(np.abs(got - want)))}}))
"""


@pytest.mark.parametrize("case,tree_min", [(("bunny", 96, 54, 4, 6), 300), (("bunny4", 64, 36, 2, 6), 200)])
def test_coop_tree_more_leaves(case, tree_min):
    env = dict(os.environ, RT_LEAF_TREE_MIN=str(tree_min))
    code = CHILD.format(tests=os.path.dirname(os.path.abspath(__file__)), root=T.ROOT, case=case)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["tree_nodes"] > 0, "the lowered threshold did not produce leaf trees"
    assert r["same"], f"max |GPU - oracle| = {r['maxdiff']}"

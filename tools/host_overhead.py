"""Host-side cost of one rt_render call (argument checks + launch), tiny frame, N calls."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

rt = G.load_package()
torch.cuda.set_device(0)
w, h = 16, 16
s = rt.Scene()
s.setup("bunny")
s.set_viewport(w, h)
rng = rt.alloc_rng(w * h)
rt.init_rng_states(rng, w, h, 1)
s.upload(rng.data_ptr())
a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
for _ in range(10):
    rt.render(s, a, b, w, h, 1, 1)
torch.cuda.synchronize()
n = 200
t = time.perf_counter()
for _ in range(n):
    rt.render(s, a, b, w, h, 1, 1)
host = (time.perf_counter() - t) / n
torch.cuda.synchronize()
print(f"rt_render host call: {host * 1e6:.1f} us")

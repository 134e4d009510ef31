"""Multi-GPU frame sharding.

Every pixel owns its RNG subsequence (curand_init(seed, y*W + x), Random.cu:7), so any pixel
partition renders bit-identical pixels.  The frame is cut into 16x16 tiles (the reference's
launch blocks, main_raytracing.cu:207-210) dealt round-robin over the ranks: rank r renders
tiles r, r + N, r + 2N, ... into a compact shard [k][256] of float4 (slot = k*256 + tid), one
gather over RCCL (xGMI) brings the N shards to rank 0, and rt_unshard scatters them back into
the pitched surface.

Plans: round-robin (above) or cost-aware (rt_shard_plan: longest processing time first from a
probe frame's per-wave clocks, every rank's heaviest tiles first), passed to the kernels as tile
lists.  The gather is rt_gather_shards (RCCL, librt_hip.so) on the GPU box; ``gather_shards``
below is the torch.distributed form used by the gloo rehearsal on CPU.

This module holds the host-side bookkeeping used by bench.py and the gloo tests; the data path
itself (render into shards, gather, unshard) is the HIP kernels and RCCL behind the C-ABI.
"""
import numpy as np

TILE = 16
TILE_PIXELS = TILE * TILE


def tiles_total(width, height):
    return ((width + TILE - 1) // TILE) * ((height + TILE - 1) // TILE)


def tiles_of_shard(width, height, shard_index, shard_count):
    """Tiles rank `shard_index` renders (rt_shard_tiles restated)."""
    t = tiles_total(width, height)
    if shard_index >= t:
        return 0
    return (t - shard_index + shard_count - 1) // shard_count


def slot_pixels(width, height, shard_index, shard_count, per_shard=None, tile_list=None):
    """(x, y) of every slot of a compact shard, -1 for padding slots.

    Slot k*256 + tid holds tile shard_index + k*shard_count (or tile_list[k] for an explicit
    plan, rt_shard_plan; entries < 0 are padding); within a tile, wave w = tid >> 6 covers the
    8x8 sub-tile ((w & 1) * 8, (w >> 1) * 8) and lane l = tid & 63 the pixel (l & 7, l >> 3) of
    it (rt_common.h tile_pixel)."""
    if tile_list is not None:
        tile_list = np.asarray(tile_list)
        k = len(tile_list)
    else:
        k = tiles_of_shard(width, height, shard_index, shard_count)
    per_shard = k if per_shard is None else per_shard
    tiles_x = (width + TILE - 1) // TILE
    tid = np.arange(TILE_PIXELS)
    w, l = tid >> 6, tid & 63
    lx = (w & 1) * 8 + (l & 7)
    ly = (w >> 1) * 8 + (l >> 3)
    xs = np.full((per_shard, TILE_PIXELS), -1, dtype=np.int64)
    ys = np.full((per_shard, TILE_PIXELS), -1, dtype=np.int64)
    for j in range(k):
        tile = int(tile_list[j]) if tile_list is not None else shard_index + j * shard_count
        if tile < 0:
            continue
        x = (tile % tiles_x) * TILE + lx
        y = (tile // tiles_x) * TILE + ly
        ok = (x < width) & (y < height)
        xs[j] = np.where(ok, x, -1)
        ys[j] = np.where(ok, y, -1)
    return xs.reshape(-1), ys.reshape(-1)


def gather_shards(shard, rank, world, out=None):
    """One collective: every rank's compact shard [per_shard*256, 4] to rank 0 (dist.gather;
    RCCL over xGMI on the GPU box, gloo in the CPU tests).  Returns the [world, ...] stack on
    rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    if shard.is_cuda and dist.get_backend() == "gloo":
        # rehearsal of the multi-GPU path on one box (gloo gathers host tensors): stage via host
        got = gather_shards(shard.cpu(), rank, world)
        if rank != 0:
            return None
        if out is None:
            out = torch.empty((world,) + tuple(shard.shape), dtype=shard.dtype, device=shard.device)
        out.copy_(got)
        return out
    if rank == 0:
        if out is None:
            out = torch.empty((world,) + tuple(shard.shape), dtype=shard.dtype, device=shard.device)
        dist.gather(shard, list(out.unbind(0)), dst=0)
        return out
    dist.gather(shard, None, dst=0)
    return None

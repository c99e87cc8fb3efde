"""Multi-GPU frame rendering.

Two decompositions of one frame over the ranks of the default process group:

* tile sharding (default in bench.py): the frame's 8x8 tiles are dealt out
  round-robin, tile t to rank t % world, so cheap (sky) and expensive tiles
  spread evenly; each rank renders ALL strata of its tiles into a compact tile
  buffer (RT_LAYOUT_TILES), adds each tile's chunk partials on its device
  (rt_tiles_sum_device), and rank 0 gathers the tile sums (1/world of the frame
  from each rank, over all of rank 0's xGMI links at once) and reorders them
  into the frame on its device (rt_tiles_to_frame_device): the timed region
  runs library kernels and the RCCL gather, no framework ops.
  Every pixel is computed by exactly one GPU.  A rank's work units are the
  library's (strata_chunks = RT_CHUNKS_AUTO: head chunks sized to the strata,
  the last tiles in finer chunks, the chunk sum inside the call), or every
  tile in `auto_chunks` chunks when a unit target is given.  Either split
  groups a pixel's strata differently from the one-GPU frame launch (but for
  a rank holding more than 4 tiles per wave slot, which takes the frame plan),
  so the frame equals the one-GPU frame up to fp64 summation order (the 2-rank
  rehearsal measures ~1e-14).  The C ABI's rt_multi_render (strata_chunks 0)
  keeps the frame launch's split and is bit-identical.
* stratum sharding (below): ranks split the strata and reduce(sum) full-frame
  accumulators — the SURVEY §8(e) recommendation; it moves ~2x the frame per
  rank through a ring and changes the fp64 summation order.

The reference is single-GPU (no NCCL/MPI).  Here a frame's strata
(the sqrt(spp) x sqrt(spp) grid of StaticCamera.cpp:74-76, linear index
s_j*sqrt_spp + s_i) are split into contiguous ranges, one per rank; every rank
renders ALL pixels for its range into its own fp64 sum buffer (RT_OUT_SUM), and a
single reduce(sum) to rank 0 combines them — over RCCL/xGMI for GPU ranks, over
gloo for the CPU tests.  The counter-based RNG is keyed by the global stratum
index, so the union of the shards is exactly the one-GPU sample set: the result
equals a single-GPU render up to fp64 summation order.
"""
import ctypes as C
import os

import torch
import torch.distributed as dist

from . import abi


def strata_shard(n_strata, rank, world):
    """Contiguous stratum range [begin, end) of `rank` (balanced to within one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return (rank * n_strata // world, (rank + 1) * n_strata // world)


def reduce_frame(acc, dst=0):
    """Sum every rank's accumulator into `dst` (in place on dst)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(acc, dst=dst, op=dist.ReduceOp.SUM)
    return acc


class ShardedRenderer:
    """Renders one frame per call across the ranks of the default process group.

    render_fn(frame, acc, seed, strata=(begin, count)) must overwrite `acc` with
    the raw per-pixel sums of that stratum range (the Renderer.render_device
    contract with output=RT_OUT_SUM, accumulate=0)."""

    def __init__(self, render_fn, frame, rank=0, world=1):
        self.render_fn = render_fn
        self.frame = frame
        self.rank, self.world = rank, world
        n = frame.sqrt_spp * frame.sqrt_spp
        self.strata = strata_shard(n, rank, world)

    def step(self, acc, seed):
        b, e = self.strata
        self.render_fn(self.frame, acc, seed, (b, e - b))
        return reduce_frame(acc)

    def image(self, acc):
        """Scaled radiance on rank 0 (pixel_samples_scale * sum)."""
        return acc * self.frame.pixel_samples_scale


def tile_counts(frame, world):
    """(tiles in the frame, tiles per rank padded to the largest shard)."""
    n = ((frame.image_width + 7) // 8) * ((frame.image_height + 7) // 8)
    return n, (n + world - 1) // world


def _stream_of(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def device_tiles_sum(parts, out):
    """Chunk partials [T, chunks, 64, 3] -> tile sums `out` [T, 64, 3] on the
    device (rt_tiles_sum_device: chunk order, the one-GPU frame launch's
    summation order), on the tensors' current stream."""
    from .lib import check, load
    assert parts.is_cuda and out.is_cuda and parts.is_contiguous() and out.is_contiguous()
    assert parts.dtype == out.dtype == torch.float64 and out.shape == (parts.shape[0], 64, 3)
    check(load().rt_tiles_sum_device(C.c_void_p(parts.data_ptr()), parts.shape[0], parts.shape[1],
                                     C.c_void_p(out.data_ptr()), C.c_void_p(_stream_of(out))))
    return out


def device_tiles_to_frame(gathered, frame, out):
    """Gathered compact tile sums [world, T_r, 64, 3] (rank r holds tiles r,
    r + world, ... in RT_LAYOUT_TILES order) -> the frame's raw sums `out`
    [H, W, 3] on the device (rt_tiles_to_frame_device)."""
    from .lib import check, load
    from .render import Renderer
    import torch
    assert gathered.is_cuda and out.is_cuda and gathered.is_contiguous() and out.is_contiguous()
    # the kernel reads both as doubles, gathered as [world][T_r][64][3] with
    # tile t at (t % world, t // world)
    assert gathered.dtype == out.dtype == torch.float64
    assert gathered.dim() == 4 and tuple(gathered.shape[2:]) == (64, 3)
    assert out.shape == (frame.image_height, frame.image_width, 3)
    n_tiles = ((frame.image_width + 7) // 8) * ((frame.image_height + 7) // 8)
    assert gathered.shape[1] >= (n_tiles + gathered.shape[0] - 1) // gathered.shape[0]
    p = Renderer.params(output=abi.RT_OUT_SUM)
    check(load().rt_tiles_to_frame_device(C.c_void_p(gathered.data_ptr()), gathered.shape[0],
                                          gathered.shape[1], C.byref(frame), C.byref(p),
                                          C.c_void_p(out.data_ptr()), C.c_void_p(_stream_of(out))))
    return out


def host_tiles_sum(parts, out):
    """rt_tiles_sum_device's operation on host tensors (the CPU backend's
    ranks): chunk partials added in chunk order, sequentially."""
    acc = parts[:, 0].clone()
    for c in range(1, parts.shape[1]):
        acc = acc + parts[:, c]
    out.copy_(acc)
    return out


def host_tiles_to_frame(gathered, frame, out):
    """rt_tiles_to_frame_device's reorder on host tensors (the CPU backend's
    ranks): gathered [world, T_r, 64, 3], rank r holding tiles r, r + world,
    ... -> the frame's raw sums out [H, W, 3]."""
    world, t_r = gathered.shape[0], gathered.shape[1]
    W, H = frame.image_width, frame.image_height
    tx, ty = (W + 7) // 8, (H + 7) // 8
    flat = gathered.transpose(0, 1).reshape(t_r * world, 64, gathered.shape[-1])[:tx * ty]
    img = flat.reshape(ty, tx, 8, 8, -1).permute(0, 2, 1, 3, 4).reshape(ty * 8, tx * 8, -1)
    out.copy_(img[:H, :W])
    return out


def shard_units(strata):
    """Work-unit target of one rank: 32768 units (8 per wave slot) at 64 strata
    per pixel, growing with sqrt(strata / 64) up to 4x -- the fastest of the
    8-way sweeps on one GPU (profiles/r04q_shard_units_*.log,
    r04v_shard_units_*.log): C2 (64 strata) 32768, C3 (256) 65536, C4 (1024)
    and C5 (4096) 131072.  A caller overrides it through auto_chunks'
    target_units (bench.py --shard-units)."""
    return int(32768 * min(4.0, max(1.0, (strata / 64.0) ** 0.5)))


def auto_chunks(frame, world, target_units=None):
    """Stratum chunks per tile so one rank still has ~target_units wavefront work
    units (several per wave slot of the 256-CU chip): a rank of an 8-way split
    holds few tiles, and one wave per slot would make the slowest tile the
    kernel time."""
    n, t_r = tile_counts(frame, world)
    strata = frame.sqrt_spp * frame.sqrt_spp
    if target_units is None:
        target_units = shard_units(strata)
    c = max(1, min(strata, -(-target_units // max(1, t_r))))
    cs = -(-strata // c)  # strata per chunk; no empty chunks
    return -(-strata // cs)


class TileShardedRenderer:
    """Renders one frame per call with tile t on rank t % world.

    render_fn(frame, buf, seed, tiles=(first, stride), chunks) must overwrite
    `buf` with the raw sums of all strata of those tiles in RT_LAYOUT_TILES
    order (Renderer.render_device with output=RT_OUT_SUM, accumulate=0,
    layout=RT_LAYOUT_TILES, chunks=chunks): with chunks = RT_CHUNKS_AUTO (the
    default: no `chunks`, no `target_units`) `buf` is [T_r, 64, 3], the tile
    sums of the library's own work units; otherwise [T_r, chunks, 64, 3], each
    tile's strata split into `chunks`, added by tiles_sum(parts, out).  The
    chunk sum and the tile -> frame reorder are the library's device kernels
    (tiles_sum, to_frame(gathered, frame, out)); the CPU tests pass torch
    equivalents for their host tensors."""

    def __init__(self, render_fn, frame, rank=0, world=1, chunks=None, tiles_sum=None,
                 to_frame=None, target_units=None):
        self.render_fn = render_fn
        self.frame = frame
        self.rank, self.world = rank, world
        self.n_tiles, self.tiles_per_rank = tile_counts(frame, world)
        self.library_units = chunks is None and target_units is None
        if self.library_units:
            self.chunks = abi.RT_CHUNKS_AUTO
        else:
            self.chunks = auto_chunks(frame, world, target_units) if chunks is None else max(1, chunks)
        self.tiles_sum = tiles_sum or device_tiles_sum
        self.to_frame = to_frame or device_tiles_to_frame

    def on_host(self):
        """The host reorder and chunk sum (ranks on the CPU backend)."""
        self.tiles_sum, self.to_frame = host_tiles_sum, host_tiles_to_frame
        return self

    def buffer(self, device=None):
        if self.library_units:  # the tile sums themselves
            return self.sum_buffer(device)
        return torch.zeros((self.tiles_per_rank, self.chunks, 64, 3), dtype=torch.float64,
                           device=device)

    def sum_buffer(self, device=None):
        return torch.zeros((self.tiles_per_rank, 64, 3), dtype=torch.float64, device=device)

    def gather_buffer(self, device=None):
        return torch.zeros((self.world, self.tiles_per_rank, 64, 3), dtype=torch.float64,
                           device=device)

    def frame_buffer(self, device=None):
        return torch.zeros((self.frame.image_height, self.frame.image_width, 3),
                           dtype=torch.float64, device=device)

    def render(self, buf, seed, out=None):
        """Render this rank's tiles; returns the per-tile sums [T_r, 64, 3] (the
        chunk sum, in fixed chunk order) in `out` (a sum_buffer)."""
        self.render_fn(self.frame, buf, seed, (self.rank, self.world), self.chunks)
        if self.library_units:
            return buf
        if self.chunks == 1:
            return buf[:, 0]
        return self.tiles_sum(buf, out if out is not None else self.sum_buffer(buf.device))

    def gather(self, tiles, gathered=None, async_op=False):
        """Collect every rank's [T_r, 64, 3] tile sums on rank 0 (gathered:
        [world, T_r, 64, 3])."""
        if self.world == 1:
            gathered[0].copy_(tiles)
            return None
        parts = list(gathered.unbind(0)) if self.rank == 0 else None
        return dist.gather(tiles.contiguous(), gather_list=parts, dst=0, async_op=async_op)

    def frame_sums(self, gathered, out=None):
        """The frame's raw sums [H, W, 3] from the gathered tile sums."""
        return self.to_frame(gathered, self.frame,
                             out if out is not None else self.frame_buffer(gathered.device))

    def step(self, buf, gathered, seed):
        tiles = self.render(buf, seed)
        self.gather(tiles, gathered)
        return self.frame_sums(gathered) if self.rank == 0 else None


def ranks_seen(device=None):
    """Distinct rank ids the default process group's collective actually
    reached (an all_gather of every rank's id): the world the exchange ran
    over, as opposed to the world the launcher meant to start."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    ws = dist.get_world_size()
    mine = torch.tensor([dist.get_rank()], dtype=torch.int64, device=device)
    allv = [torch.zeros_like(mine) for _ in range(ws)]
    dist.all_gather(allv, mine)
    return len({int(v.item()) for v in allv})


def max_over_ranks(value, device=None):
    """Max of a float across ranks (the bench's timing rule)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

"""Persistent waves (rt_kernel.hip render_tiles<.., PC=true>): for chunked
frame launches of the plain BVH feature sets, a grid of resident blocks whose
waves pull (tile, stratum chunk) units from a device counter.  Small test
frames have fewer units than resident waves, so they would never take that
path; rt_tuning.grid_cap shrinks the grid to a few blocks so every wave renders many
units.  The frame must be bit-identical to the one-unit-per-wave launch (the
partial sums are added in chunk order either way) and match the oracle."""
import os

import numpy as np
import pytest

from rtx.render import Renderer, camera_frame
from rtx.scene import load_scene
import oracle_lib as O

pytestmark = pytest.mark.gpu
SCENES = os.path.join(O.ROOT, "real-time-ray-tracing-engine_amd", "scenes")


def _render(S, f, seed, tuning):
    with Renderer(S, tuning=tuning) as R:
        return R.render(f, seed=seed)


@pytest.mark.parametrize("name,arity,cap,pcw", [("bouncing_seed42", 2, 1, 16), ("bouncing_seed42", 2, 3, 16),
                                                ("bouncing_seed42", 4, 2, 16), ("bouncing_seed42", 2, 3, 4),
                                                ("bouncing_seed42", 4, 5, 4)])
def test_persistent_waves_match_one_unit_per_wave(name, arity, cap, pcw):
    """pcw: waves per persistent block -- 16 (one block per CU owning its LDS:
    the whole tree, items and spheres staged) or 4 (the fallback for traversal
    stacks too deep for 16 waves, forced here by rt_tuning.pc_waves)."""
    S = load_scene(os.path.join(SCENES, name + ".json"))
    S.bvh_arity = arity
    cam = S.camera_desc(image_width=64, samples_per_pixel=16, max_depth=8)
    f = camera_frame(cam)
    with Renderer(S, tuning={"grid_cap": cap, "pc_waves": pcw if pcw == 4 else 0}) as R:
        info = R.info()
        pers = R.render(f, seed=5)
    assert info["persistent_block_waves"] == pcw
    if pcw == 16 and arity == 2:  # C3's scene: everything staged
        assert info["lds_nodes_persistent"] == info["n_nodes"] and info["lds_prims_persistent"] == 1
    single = _render(S, f, 5, {"grid_cap": 1000000})  # cap above the block count: one unit per wave
    assert np.array_equal(pers, single)
    ref = O.oracle_render(S, cam, O.MODE_COUNTER, 5)
    assert np.abs(pers - ref).max() <= 1e-4


@pytest.mark.parametrize("layout_chunks", [1, 4])
def test_persistent_tile_subset_launch(layout_chunks):
    """Tile-subset launches (a multi-GPU rank's tiles t = 1 (mod 3), compact
    RT_LAYOUT_TILES output, optionally stratum chunks) also run persistent when
    they have more units than resident waves: bit-identical to one unit per
    wave."""
    from rtx import abi
    S = load_scene(os.path.join(SCENES, "bouncing_seed42.json"))
    cam = S.camera_desc(image_width=64, samples_per_pixel=16, max_depth=8)
    f = camera_frame(cam)

    def run(cap):
        with Renderer(S, tuning={"grid_cap": cap}) as R:
            return R.render(f, seed=8, output=abi.RT_OUT_SUM, tiles=(1, 3),
                            layout=abi.RT_LAYOUT_TILES, chunks=layout_chunks)
    pers, single = run(1), run(1000000)
    assert np.array_equal(pers, single)
    assert pers.any()


def test_staged_tree_forms_render_the_same_frame():
    """C3's scene in the persistent instance with the whole tree staged in LDS
    (80-B DNodeL nodes, child entries as byte offsets, the sign-picked visit),
    with only a prefix staged (DNodeL prefix + DNode table in HBM, the min/max
    visit) and with nothing staged: the three walks visit the same nodes in the
    same order (the sign-picked planes ARE the min/max picks, rt_path.h), so
    the frames are bit-identical -- and match the oracle."""
    S = load_scene(os.path.join(SCENES, "bouncing_seed42.json"))
    cam = S.camera_desc(image_width=64, samples_per_pixel=16, max_depth=8)
    f = camera_frame(cam)
    frames, infos = {}, {}
    for staged in ("all", "100", "0"):
        tune = {"grid_cap": 3}
        if staged != "all":  # rt_tuning.lds_nodes_pc: at most N nodes, < 0 none
            tune["lds_nodes_pc"] = int(staged) if int(staged) > 0 else -1
        with Renderer(S, tuning=tune) as R:
            infos[staged] = R.info()
            frames[staged] = R.render(f, seed=9)
    assert infos["all"]["lds_nodes_persistent"] == infos["all"]["n_nodes"]
    assert infos["100"]["lds_nodes_persistent"] == 100 and infos["0"]["lds_nodes_persistent"] == 0
    assert np.array_equal(frames["all"], frames["100"])
    assert np.array_equal(frames["all"], frames["0"])
    ref = O.oracle_render(S, cam, O.MODE_COUNTER, 9)
    assert np.abs(frames["all"] - ref).max() <= 1e-4

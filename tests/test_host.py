"""CPU tests: C-ABI library load + exports, host-side logic (clip plans, weights, checkpoints, EF),
and the multi-rank clip sharding over gloo (world_size 2 and 3)."""
import ctypes
import os
import re
import socket

import numpy as np
import pytest
import torch

from tests.conftest import REPO, golden

HEADER = os.path.join(REPO, "include", "clasfv.h")


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int64_t|int|void)\s+\*?(clasfv_\w+)\s*\(", txt, re.M)))


def test_library_builds_and_exports_every_header_symbol():
    from clasfv_amd import _lib
    from clasfv_amd.build import build
    path = build()
    assert os.path.exists(path)
    lib = ctypes.CDLL(path)
    funcs = header_functions()
    assert len(funcs) >= 14
    for f in funcs:
        assert hasattr(lib, f), f"{f} declared in include/clasfv.h but not exported"
    assert set(funcs) == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/clasfv.h"


def test_abi_version_matches_header():
    from clasfv_amd import _lib
    m = re.search(r"#define CLASFV_ABI_VERSION (\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == _lib.ABI_VERSION == _lib.load().clasfv_version()
    bits = dict(re.findall(r"CLASFV_VARIANT_(\w+) = (\d+)", open(HEADER).read()))
    assert {k.lower(): int(v) for k, v in bits.items()} == _lib.VARIANTS


def test_library_reports_errors_without_gpu():
    from clasfv_amd import _lib
    lib = _lib.load()
    assert lib.clasfv_version() == _lib.ABI_VERSION
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = lib.clasfv_create(0, ctypes.byref(h))
    assert rc != 0 and lib.clasfv_last_error()
    assert lib.clasfv_forward(None, None, 1, 32, 112, 112, None, None, None) == -1  # CLASFV_EINVAL


def test_product_path_has_no_oracle_or_cpu_fallback():
    pkg = os.path.join(REPO, "fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "oracle" not in re.sub(r'""".*?"""', "", src, flags=re.S).replace("# ", ""), f


def test_arch_spec_matches_reference_counts():
    import clasfv_amd.arch as A
    spec = A.state_dict_spec()
    assert len(spec) == 242
    assert A.count_parameters(spec) == A.NUM_PARAMS_REFERENCE
    mids = [c.cout for r, c in A.backbone_convs() if r == "sp1"]
    assert mids == [144, 144, 230, 288, 460, 576, 921, 1152]
    assert sum(1 for k in spec if k.endswith("num_batches_tracked")) == 39


def test_synthetic_weights_deterministic():
    import clasfv_amd.weights as W
    a = W.synthetic_state_dict(7)
    b = W.synthetic_state_dict(7)
    c = W.synthetic_state_dict(8)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    assert not np.array_equal(a["comb_1_layer.weight"], c["comb_1_layer.weight"])
    assert all(v.dtype == np.float32 for k, v in a.items() if not k.endswith("num_batches_tracked"))


def test_checkpoint_roundtrip_with_module_prefix(tmp_path):
    import clasfv_amd.weights as W
    sd = W.synthetic_state_dict(3)
    p = str(tmp_path / "ckpt.pth")
    W.save_checkpoint(p, sd, module_prefix=True)
    raw = torch.load(p, weights_only=True)
    assert next(iter(raw["model"])).startswith("module.")
    back = W.load_checkpoint(p)
    assert list(back) == list(sd) and all(np.array_equal(back[k], sd[k]) for k in sd)


@pytest.mark.parametrize("T", [33, 40, 47, 48, 64, 70, 80, 100, 199, 200, 256])
@pytest.mark.parametrize("f,step", [(1, 1), (5, 1), (3, 2), (10, 1), (5, 3)])
def test_clip_plan_matches_oracle(T, f, step):
    from clasfv_amd import fuse_utils as FU
    from oracle import fuse_ref
    k = FU.clamp_num_clips(T, f, step)
    assert k == fuse_ref.clamp_num_clips(T, f, step)
    if k == 0:
        return
    table, clip0 = FU.clip_table(T, k, step)
    for j in range(k):
        n_ref = len(range(0, fuse_ref.n_clip_frames(T - j * step), 32))
        nxt = clip0[j + 1] if j + 1 < k else len(table)
        assert nxt - clip0[j] == n_ref
        assert all(s == j * step for s, _ in table[clip0[j]:nxt])


def test_ef_matches_reference_golden():
    from clasfv_amd.echo import compute_ef_using_putative_clips, get2dPucks
    g = golden("ef.npz")
    for name in g["names"]:
        shp = tuple(g[name + "_shape"])
        m = np.unpackbits(g[name + "_bits"])[: int(np.prod(shp))].reshape(shp).astype(np.int64)
        efs, pairs = compute_ef_using_putative_clips(m, name, return_edes=True)
        assert np.array(pairs, np.int64).reshape(-1, 2).tolist() == g[name + "_pairs"].tolist(), name
        np.testing.assert_allclose(np.array(efs, np.float64), g[name + "_efs"], rtol=0, atol=1e-9, equal_nan=True)
    fr = np.unpackbits(g["pucks_frames"]).reshape(-1, 112, 112)
    for i, f in enumerate(fr):
        L, R = get2dPucks(f.astype(int), (1.0, 1.0))
        assert L == g["pucks_L"][i]
        np.testing.assert_array_equal(R, g["pucks_R"][i])
    # SURVEY §8c known answer: four ED-ES pairs of the pulsing ellipse, EF 68.808074 each
    np.testing.assert_allclose(g["ellipse200_efs"], 68.808074, atol=1e-6)


def test_synthetic_video_and_lv_masks():
    import clasfv_amd.synthetic as S
    v = S.echo_video_uint8(60, seed=0)
    assert v.shape == (60, 112, 112, 3) and v.dtype == np.uint8
    assert np.array_equal(v[..., 0], v[..., 2])
    m = S.ellipse_masks(60)
    area = m.sum((1, 2))
    assert area.argmax() in (0, 50) and abs(int(area.argmin()) - 25) <= 1


def test_shard_bounds_partition():
    from clasfv_amd.dist import shard_bounds
    for n in (0, 1, 7, 30, 31, 384, 1920):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, n_total, q):
    import torch.distributed as dist
    from clasfv_amd.dist import run_clip_shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def compute(lo, hi):  # stand-in per-clip "logits": a function of the global clip index only
            idx = torch.arange(lo, hi, dtype=torch.float32)
            return idx[:, None, None] * 10 + torch.arange(6, dtype=torch.float32).view(1, 2, 3)
        out = run_clip_shard(n_total, rank, world, compute, torch.empty((0, 2, 3)))
        q.put((rank, out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 30), (2, 1), (3, 31), (2, 0)])
def test_clip_shard_all_gather_gloo(world, n_total):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ref = np.arange(n_total, dtype=np.float32)[:, None, None] * 10 + np.arange(6, dtype=np.float32).reshape(1, 2, 3)
    for r in range(world):
        np.testing.assert_array_equal(res[r], ref)


def _plans(sizes):
    out, off = [], 0
    for n in sizes:
        out.append({"n": n, "offset": off})
        off += n
    return out


def _owner_worker(rank, world, port, sizes, q):
    import torch.distributed as dist
    from clasfv_amd.dist import exchange_to_owners, owner_of_clips, shard_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        owners = owner_of_clips(_plans(sizes), world)
        lo, hi = shard_bounds(len(owners), rank, world)
        local = torch.arange(lo, hi, dtype=torch.float32)[:, None] * torch.ones(1, 3)  # row g = g
        got = exchange_to_owners(local, owners, rank, world)
        q.put((rank, got.numpy(), got.data_ptr() == local.data_ptr()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes", [(2, [6, 5, 7]), (3, [1, 1, 1, 1, 1]), (2, [30, 30]), (3, [4, 0, 9, 2]),
                                         (2, [30] * 16), (3, [7, 30, 2, 30, 11])])
def test_owner_exchange_gloo(world, sizes):
    """Owner exchange (all_to_all of per-clip rows to the rank fusing their video): every rank gets
    exactly the rows of the videos it owns (video_owners), in global order; when every video lies in
    one rank's block (e.g. 8 equal videos per rank) nothing moves and each rank keeps its own rows."""
    import torch.multiprocessing as mp
    from clasfv_amd.dist import rows_exchanged, owner_of_clips, video_owners
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, rows, same = q.get(timeout=120)
        res[r] = (rows, same)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    offs = np.cumsum([0] + sizes)
    vown = video_owners(_plans(sizes), world)
    moved = rows_exchanged(owner_of_clips(_plans(sizes), world), world)
    for r in range(world):
        want = np.concatenate([np.arange(offs[v], offs[v + 1]) for v in range(len(sizes)) if vown[v] == r] or
                              [np.zeros(0)]).astype(np.float32)
        np.testing.assert_array_equal(res[r][0][:, 0], want)
        if moved == 0 and len(want):
            assert res[r][1], "no exchange: the rank's own rows are returned as they are"
    if sizes == [30] * 16:
        assert moved == 0


def test_owner_mapping_is_block_aligned():
    """SURVEY 8(e) / config[2]: 64 equal videos over 8 ranks (and 8 per rank over 2) exchange no
    clip; a straddling video is owned by the rank holding most of its clips."""
    from clasfv_amd.dist import owner_of_clips, rows_exchanged, video_owners
    for world, n_vid in ((8, 64), (2, 16), (4, 64), (8, 8), (1, 5)):
        plans = _plans([30] * n_vid)
        assert rows_exchanged(owner_of_clips(plans, world), world) == 0
        assert video_owners(plans, world) == [v * world // n_vid for v in range(n_vid)]
    # 3 videos of 30 clips over 2 ranks: blocks [0,45), [45,90) -> video 1 straddles 15/15 -> rank 0
    plans = _plans([30, 30, 30])
    assert video_owners(plans, 2) == [0, 0, 1]
    assert rows_exchanged(owner_of_clips(plans, 2), 2) == 15
    plans = _plans([10, 40, 10])  # blocks [0,30), [30,60): video 1 has 20 clips in rank 0, 20 in 1 -> 0
    assert video_owners(plans, 2) == [0, 0, 1]


def test_fast_division_magic_numbers(tmp_path):
    """FastDiv (csrc/common.h), the multiply-high division the conv kernels decode tile indices with,
    equals integer division for every divisor < 5000 and the engine's map sizes (tools/fastdiv_check.cpp
    restates the same construction on the host)."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    src = os.path.join(REPO, "tools", "fastdiv_check.cpp")
    exe = str(tmp_path / "fdc")
    subprocess.run([gxx, "-O2", "-std=c++17", src, "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and "mismatches: 0" in r.stdout, r.stdout + r.stderr
    hdr = open(os.path.join(REPO, "fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking_amd",
                            "csrc", "common.h")).read()
    assert "(((1ull << 32) * ((1ull << l) - d)) / d + 1)" in hdr  # the construction the check restates


def test_wino4w_inline_asm_accumulators_untouched(tmp_path):
    """conv_wino4w's N tiles past W4W_NTA accumulate in VGPRs through inline-asm MFMAs that hipcc
    neither models nor pads: the product build is safe only while no compiler instruction in the
    chunk loop (or between the loop exit and the 12-state drain) touches those registers and the
    kernel has no scratch. tools/audit_wino4w_asm.py checks that on the device assembly of every
    conv_wino4w instantiation (and flags an injected v_mov into an accumulator)."""
    import shutil
    import sys
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc) and shutil.which("hipcc") is None:
        pytest.skip("hipcc not available")
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import audit_wino4w_asm as A
    path = A.compile_asm(out_dir=str(tmp_path))
    problems, n = A.audit(path)
    assert n >= 8 and problems == [], problems
    # the audit sees a violation: a compiler copy into the first asm accumulator inside the loop
    lines = open(path).read().splitlines()
    k = next(i for i, ln in enumerate(lines) if "v_mfma_f32_16x16x4_f32 v[" in ln)
    acc = int(re.search(r"v\[(\d+):", lines[k]).group(1))
    j = next(i for i in range(k, 0, -1) if ";;#ASMSTART" in lines[i])
    lines.insert(j, f"\tv_mov_b32 v{acc}, 0")
    bad = tmp_path / "bad.s"
    bad.write_text("\n".join(lines))
    problems, _ = A.audit(str(bad))
    assert len(problems) == 1 and f"v{acc}" in problems[0]


def test_strict_reference_clamp_and_frames():
    """src/fuse_utils.py:38-42 clamps T in [32, 32 + step) to K = 0 (then IndexError at :82);
    strict_reference=False runs one pass there, and keeps all T frames for step > 1 (:85)."""
    from clasfv_amd import fuse_utils as FU
    assert FU.clamp_num_clips(32, 1, 1) == 0 and FU.clamp_num_clips(32, 1, 1, strict_reference=False) == 1
    assert FU.clamp_num_clips(34, 5, 3) == 0 and FU.clamp_num_clips(34, 5, 3, strict_reference=False) == 1
    assert FU.clamp_num_clips(200, 5, 1, strict_reference=False) == 5
    assert FU.fused_frames(80, 2) == 79 and FU.fused_frames(80, 2, strict_reference=False) == 80
    labels = torch.arange(3 * 6, dtype=torch.uint8).view(3, 6, 1, 1)  # 3 passes x 6 frames
    fused = torch.tensor([100, 101, 102, 103], dtype=torch.uint8).view(4, 1, 1)  # frames 0, 3, 4, 5
    got = FU.keep_dropped_frames(labels, fused, 3).view(-1).tolist()
    assert got == [100, 1, 2, 101, 102, 103]


def test_config2_plan_videos_per_rank_and_no_exchange():
    """BASELINE config[2]: 64 x 200-frame videos over 8 ranks (f = 1 and f = 5): every rank holds
    exactly its 8 videos and no clip crosses ranks."""
    from clasfv_amd.dist import exchange_stats, videos_needed
    lengths = [200] * 64
    for f in (1, 5):
        for world in (1, 2, 4, 8):
            need = [videos_needed(lengths, f, 1, r, world) for r in range(world)]
            assert [len(n) for n in need] == [64 // world] * world
            assert sorted(sum(need, [])) == list(range(64))
            assert exchange_stats(lengths, f, 1, world) == (0, 0)
    rows, nbytes = exchange_stats([70, 96, 45], 3, 1, 2)
    assert rows > 0 and nbytes == rows * 32 * 112 * 112 * 4


def test_bench_rejects_world_size_mismatch():
    """bench.py under a launcher: WORLD_SIZE must equal --gpus (checked before any GPU call)."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1"], capture_output=True, text=True, timeout=120,
                       cwd=REPO, env=env)
    assert r.returncode != 0 and "must agree" in r.stderr


def test_itk_voting_oracle_rule():
    from oracle import fuse_ref
    a = np.array([[0, 1], [1, 1]], np.uint8)
    b = np.array([[0, 0], [1, 0]], np.uint8)
    c = np.array([[1, 0], [1, 1]], np.uint8)
    np.testing.assert_array_equal(fuse_ref.itk_voting([a, b]), [[0, 2], [1, 2]])  # ties -> undecided (max + 1)
    np.testing.assert_array_equal(fuse_ref.itk_voting([a, b, c]), [[0, 0], [1, 1]])
    np.testing.assert_array_equal(fuse_ref.majority_vote([a, b]), [[0, 0], [1, 0]])


def test_echo_weights_keep_the_random_recipe_elsewhere():
    """The "echo" recipe changes only its designed units; every other weight is the random recipe's."""
    import clasfv_amd.weights as W
    r, e = W.synthetic_state_dict(1234), W.echo_state_dict(1234)
    assert list(r) == list(e)
    same = [k for k in r if np.array_equal(r[k], e[k])]
    assert len(same) > 150
    for k in ("r2plus1d_model.layer2.0.conv1.0.0.weight", "r2plus1d_model.layer4.1.conv2.0.3.weight"):
        assert np.array_equal(r[k], e[k])
    w = e["r2plus1d_model.stem.0.weight"]
    assert np.array_equal(w[6:], r["r2plus1d_model.stem.0.weight"][6:])
    assert np.allclose(w[0].sum(), W.ECHO["S0"])  # box mean of the intensity
    w1 = e["comb_1_layer.weight"].reshape(64, 1024)
    assert np.array_equal(w1[7:], r["comb_1_layer.weight"].reshape(64, 1024)[7:])

"""Host-side logic that needs no GPU: checkpoint metrics with numpy values, the
bench's multi-rank launch path (`bench.py --gpus 2` spawns torch.distributed.run ranks), and
the drop-threshold encoding the C header documents."""
import json
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_checkpoint_roundtrip_with_numpy_metrics(tmp_path):
    """run_evaluate-style metrics (numpy int64 predictions, numpy float scores) survive
    save_checkpoint -> load_checkpoint(weights_only=True); a file written the reference's way
    (numpy scalars pickled as-is, `train/train_latent_vit_v2.py:168,181`) loads too."""
    from fervit.checkpoint import load_checkpoint, save_checkpoint

    m = torch.nn.Linear(4, 3)
    metrics = {"val_f1": np.float64(0.5), "predictions": list(np.array([1, 2, 3], dtype=np.int64)),
               "labels": np.array([0, 2, 3])}
    p = str(tmp_path / "a.pt")
    save_checkpoint(p, m, torch.optim.AdamW(m.parameters()), 3, metrics=metrics, config={"model": "x"})
    ck = load_checkpoint(p, model=m)
    assert ck["metrics"]["predictions"] == [1, 2, 3] and type(ck["metrics"]["predictions"][0]) is int
    assert ck["metrics"]["labels"] == [0, 2, 3] and ck["metrics"]["val_f1"] == 0.5
    # reference-style file: numpy scalars stored raw (legacy serialization)
    q = str(tmp_path / "ref.pt")
    torch.save({"epoch": 1, "model_state_dict": m.state_dict(), "metrics": metrics}, q,
               _use_new_zipfile_serialization=False)
    ck = load_checkpoint(q, model=m)
    assert [int(v) for v in ck["metrics"]["predictions"]] == [1, 2, 3]
    # numpy 1.x module path of the scalar reconstructor
    raw = open(q, "rb").read().replace(b"numpy._core.multiarray", b"numpy.core.multiarray")
    r = str(tmp_path / "ref_np1.pt")
    open(r, "wb").write(raw)
    ck = load_checkpoint(r, model=m)
    assert float(ck["metrics"]["val_f1"]) == 0.5


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` outside torch.distributed starts 2 ranks (gloo dry run on CPU) and
    reports what the ranks saw."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, timeout=240, cwd=ROOT)
    out = r.stdout.decode(errors="replace")
    assert r.returncode == 0, out[-2000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, timeout=120, cwd=ROOT)
    assert r.returncode != 0 and b"WORLD_SIZE=1" in r.stdout


def test_drop_threshold_encoding():
    """include/fervit.h: thresh = round(p * 65536) in [1, 65535] for 0 < p < 1, 0 = off,
    65536 = drop all (scale 0)."""
    from fervit.ops import drop_args

    assert drop_args(0.0) == (0, 1.0)
    assert drop_args(0.1) == (6554, 1.0 / 0.9)
    assert drop_args(1e-9)[0] == 1 and drop_args(1 - 1e-9)[0] == 65535
    assert drop_args(1.0) == (65536, 0.0)

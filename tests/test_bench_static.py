"""bench.py's N > 1 lines: every collective (gloo all-reduce / all-gather /
barrier) must run on every rank, so none may follow the point where the other
ranks return and rank 0 alone writes the JSON line.  (Round 3 found C5's
second-round summary all-reduces after that point: N = 2 ended with
"connection closed by peer".)"""
import ast
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COLLECTIVES = {"allsum", "allmax", "allgather_int", "barrier", "all_reduce", "all_gather",
               "broadcast", "second_round"}


def _is_rank0_return(node):
    """`if rank != 0: return`"""
    if not isinstance(node, ast.If) or not node.body or not isinstance(node.body[0], ast.Return):
        return False
    t = node.test
    return (isinstance(t, ast.Compare) and isinstance(t.left, ast.Name) and t.left.id == "rank"
            and isinstance(t.ops[0], ast.NotEq))


def _called_names(node):
    for n in ast.walk(node):
        if isinstance(n, ast.Call):
            f = n.func
            if isinstance(f, ast.Name):
                yield f.id
            elif isinstance(f, ast.Attribute):
                yield f.attr


def test_no_collective_after_rank0_return():
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    checked = 0
    for fn in ast.walk(tree):
        if not isinstance(fn, ast.FunctionDef):
            continue
        for i, stmt in enumerate(fn.body):
            if _is_rank0_return(stmt):
                checked += 1
                late = {name for s in fn.body[i + 1:] for name in _called_names(s)} & COLLECTIVES
                assert not late, f"{fn.name}: {sorted(late)} after `if rank != 0: return`"
    assert checked >= 2  # main's headline line and run_c5's line


def _run_bench(args, env_extra=None, timeout=120):
    import json
    import subprocess
    import sys
    env = {kk: v for kk, v in os.environ.items()
           if kk not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NBKD_BENCH_SAME_DEVICE")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, [json.loads(ln) for ln in lines], p.stderr


def test_gpus_n_without_launcher_starts_n_ranks():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts two ranks itself
    (torch.distributed.run children; the parent never execs) and forwards rank
    0's one JSON line: the --launch-probe ranks meet over gloo without a GPU."""
    rc, lines, err = _run_bench(["--gpus", "2", "--launch-probe"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks"] == [0, 1]


def test_gpus_n_with_fewer_gpus_fails_cleanly():
    """Fewer visible GPUs than --gpus (none here): a non-zero exit and no JSON
    line, never an n_gpus: 1 line for an N = 2 request."""
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip("two GPUs are visible")
    rc, lines, err = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert rc != 0 and not lines
    assert "GPU(s) visible" in err


def test_pmc_lookups_match_the_library_sha(tmp_path, monkeypatch):
    """roofline.traffic / step_traffic come only from a PMC summary whose
    lib_sha256 is the loaded library's (no GPU: the lookups read files)."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha256", lambda: "abc")
    json.dump({"lib_sha256": "abc", "n_particles": 100, "k": 32, "hbm_bytes_per_step": 7.0},
              open(prof / "r99_pmc_step.json", "w"))
    json.dump({"lib_sha256": "zzz", "n_particles": 100, "k": 32, "hbm_bytes_per_step": 9.0},
              open(prof / "r98_pmc_step.json", "w"))
    assert bench.pmc_step_traffic(100, 32) == (7.0, "profiles/r99_pmc_step.json")
    assert bench.pmc_step_traffic(100, 16) == (None, None)
    monkeypatch.setattr(bench, "lib_sha256", lambda: "other")
    assert bench.pmc_step_traffic(100, 32) == (None, None)
    r = bench.roofline_entry(8e9, "x", 2.0, 1000.0, step_traffic=1.0)
    assert abs(r["frac"] - 8e9 / 2e-3 / 1e9 / 8000.0) < 1e-12 and r["frac"] <= 1.0

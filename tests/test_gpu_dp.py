"""Data-parallel training step on the GPU: 2 gloo ranks sharing the card run
the benchmark's HipTrainer (graph-captured step, split backward, bucketed gradient all-reduce on
the side stream) for 2 eager + 3 replayed steps; the result must equal the step's definition
run in one process -- per-rank fwd+bwd at batch 32, gradients averaged, one AdamW + EMA update
(tools/dp_check.py).  Reference: Lightning DDP mean all-reduce (main_val.py:643-666), no SyncBN.
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, log):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", ENCDIFF_DIST_BACKEND="gloo")
    with open(log, "w") as fh:
        r = subprocess.run(cmd, cwd=REPO, env=env, stdout=fh, stderr=subprocess.STDOUT, timeout=420)
    out = open(log).read()
    assert r.returncode == 0, out[-3000:]
    return out


def test_dp_two_ranks_equal_single_process_definition(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = str(tmp_path / "dp.pt")
    tool = os.path.join(REPO, "tools", "dp_check.py")
    log = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", "29617", tool, "--mode", "dp", "--out", out],
               str(tmp_path / "dp.log"))
    print(log[-400:])
    assert "ranks_equal=True" in log
    _run([sys.executable, tool, "--mode", "w1", "--out", out + ".w1"], str(tmp_path / "w1.log"))
    r0 = torch.load(out + ".rank0", weights_only=True)
    r1 = torch.load(out + ".rank1", weights_only=True)
    w1 = torch.load(out + ".w1", weights_only=True)
    assert r0["split_lo"] is not None, "the split backward (output-block bucket overlap) did not engage"
    for k in sorted(r0["local"]):  # eager steps: what each rank sent vs its definition pass
        for r, rr in ((0, r0), (1, r1)):
            a, b = rr["local"][k].double(), w1["local"][(k, r)].double()
            print(f"step {k} rank {r}: local gradient vs definition rel-L2 "
                  f"{((a - b).norm() / b.norm()).item():.3e} bitwise={torch.equal(rr['local'][k], w1['local'][(k, r)])}")
    for k in sorted(w1["grads"]):
        g, gw = r0["grads"][k].double(), w1["grads"][k].double()
        worst = sorted(((((g[o:o + n] - gw[o:o + n]).norm() / gw[o:o + n].norm().clamp_min(1e-30)).item(), name)
                        for name, (o, sh) in w1["names"].items() for n in [int(torch.Size(sh).numel())]),
                       reverse=True)[:6]
        rel = ((g - gw).norm() / gw.norm()).item()
        print(f"step {k}: exchanged gradient vs definition rel-L2 {rel:.3e} "
              f"bitwise={torch.equal(r0['grads'][k], w1['grads'][k])} worst {worst}")
        assert rel < 1e-3, k
    for k in ("master", "exp_avg", "exp_avg_sq", "ema"):
        assert torch.equal(r0[k], r1[k]), f"ranks differ in {k}"
        d = (r0[k].double() - w1[k].double())
        rel = (d.norm() / w1[k].double().norm()).item()
        print(f"{k}: DP vs definition max-abs {d.abs().max().item():.3e} rel-L2 {rel:.3e} "
              f"bitwise={torch.equal(r0[k], w1[k])}")
        # bitwise in most runs; in a few GPU runs (two ranks + the test process on one card)
        # one rank's local gradient differed at 1e-5..1e-4 relative in its first step (DESIGN.md
        # §6), which AdamW carries forward (exp_avg reached 1.9e-4 once: the largest relative
        # parts are Encoder4 conv biases ahead of BatchNorm, whose true gradient is zero) -- far
        # below the O(1) deviation a wrong exchange (a missing bucket, a stale finalize, a wrong
        # scale) produces
        assert rel < 1e-3, k


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_dp_exchange_over_rccl_one_rank(tmp_path, wire):
    """The RCCL side of the exchange on a one-GPU box: bench.py under torch.distributed.run with
    ONE rank, backend "nccl" (= RCCL) and ENCDIFF_DP_FORCE=1, so the step runs the full DP path --
    split backward, the four captured graphs, the bucketed all-reduces (ReduceOp.AVG over the
    RCCL communicator) on the side stream with the host-issued waits.  A mean over one rank is the
    identity, so after the same steps the loss must be bitwise the plain single-process step's,
    and the JSON line must carry the exchange timing (the split engaged)."""
    import json
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    args = ["bench.py", "--batch", "32", "--steps", "4", "--warmup", "2", "--skip-cpu", "--skip-ddim"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", ENCDIFF_DP_FORCE="1")
    env.pop("ENCDIFF_DIST_BACKEND", None)
    if wire == "bf16":  # the bf16 wire format (ENCDIFF_DP_GRAD_BF16): staged, all-reduced, cast back
        env["ENCDIFF_DP_GRAD_BF16"] = "1"

    def run(cmd, log, e):
        with open(log, "w") as fh:
            r = subprocess.run(cmd, cwd=REPO, env=e, stdout=fh, stderr=subprocess.STDOUT, timeout=420)
        out = open(log).read()
        assert r.returncode == 0, out[-3000:]
        return json.loads([ln for ln in out.splitlines() if ln.startswith('{"metric"')][-1])

    dp = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
              "--master-addr", "127.0.0.1", "--master-port", "29631" if wire == "fp32" else "29633", *args],
             str(tmp_path / "rccl.log"), env)
    plain_env = dict(os.environ)
    plain_env.pop("ENCDIFF_DP_FORCE", None)
    # the DP run takes min(10, steps) extra exchange-timing steps before it reads the loss
    plain_args = [a if a != "4" else "8" for a in args]
    plain = run([sys.executable, *plain_args], str(tmp_path / "plain.log"), plain_env)
    print("RCCL one-rank exchange:", dp.get("dp"), "loss", dp["loss_simple_last"], "plain", plain["loss_simple_last"])
    assert dp.get("dp") is not None and dp["dp"]["split_backward"], dp.get("dp")
    # every coarse bucket's all-reduce was issued (timed on the exchange stream)
    assert all(b["allreduce_ms"] is not None for b in dp["dp"]["buckets"]), dp["dp"]["buckets"]
    if wire == "fp32":
        assert dp["loss_simple_last"] == plain["loss_simple_last"]
    else:  # gradients rounded to bf16 before the (identity) mean: close, not bitwise
        assert all(abs(b["wire_mb"] * 2 - b["params"] * 4 / 2 ** 20) < 0.05 for b in dp["dp"]["buckets"])
        assert abs(dp["loss_simple_last"] - plain["loss_simple_last"]) < 1e-2 * plain["loss_simple_last"]

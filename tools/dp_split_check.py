"""Data-parallel rehearsal on ONE GPU box: N ranks over gloo sharing the card (bench.py's
ENCDIFF_DIST_BACKEND=gloo mode), a few eager + graph-replayed training steps, then rank 0
prints a checksum of the parameters and the AdamW state.  Run it with ENCDIFF_DP_SPLIT=1 and
=0: the split backward only reorders launches and all-reduce buckets, so the two checksums
must be bitwise equal (and equal across repeated runs).

DP_CHECK_SAVE=<file> also saves rank 0's parameters for an element-wise comparison;
DP_CHECK_TIME=1 times each captured graph of the DP step alone (rank 0).

usage: ENCDIFF_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \
           --master-addr 127.0.0.1 --master-port 29531 tools/dp_split_check.py [--batch 64]
"""
import argparse
import hashlib
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    ws = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    dist.init_process_group(os.environ.get("ENCDIFF_DIST_BACKEND", "gloo"))
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer

    torch.manual_seed(1234)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    tr = HipTrainer(ldm, args.batch, pool_size=4096)
    tr.init_scale_factor()
    tr.capture(warmup=2)
    for _ in range(args.steps):
        tr.step()
    torch.cuda.synchronize()
    a = tr.arena
    h = hashlib.sha256()
    for buf in (a.master, a.exp_avg, a.exp_avg_sq):
        h.update(buf.detach().cpu().numpy().tobytes())
    other = [None] * ws
    dist.all_gather_object(other, h.hexdigest())
    if dist.get_rank() == 0:
        out = os.environ.get("DP_CHECK_SAVE")
        if out:
            torch.save({"master": a.master.cpu(), "exp_avg_sq": a.exp_avg_sq.cpu()}, out)
        print(f"split={os.environ.get('ENCDIFF_DP_SPLIT', '1')} split_lo={tr._split_lo} "
              f"buckets={tr.buckets.bounds} loss={tr.loss():.6f} ranks_equal={len(set(other)) == 1} "
              f"digest={other[0]}", flush=True)
    if dist.get_rank() == 0 and os.environ.get("DP_CHECK_TIME"):
        # GPU time of each captured piece of the DP step (replayed alone, rank 0)
        for name in ("_g_fb", "_g_rest", "_g_cond", "_g_opt"):
            g = getattr(tr, name)
            if g is None:
                continue
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            print(f"graph {name}: {e0.elapsed_time(e1) / 5:.3f} ms", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

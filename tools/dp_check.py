"""Data-parallel step vs its single-process definition, on ONE GPU box.

--mode dp  (under torch.distributed.run, gloo, N ranks sharing the card): every rank runs the
           bench's HipTrainer (B per rank, graph-captured step, split backward, bucketed
           all-reduce on the side stream) for `--steps` steps with its own inputs fed through
           HipTrainer.enable_feed().
--mode w1  (plain process): the definition of that DP step -- for every step, the N ranks'
           fwd+bwd at batch B one after the other on one trainer, the gradients averaged, one
           AdamW + EMA update.  (Data parallelism without SyncBN: Encoder4's BatchNorm
           statistics are per rank in both, as in the reference's Lightning DDP.)

Both save rank 0's parameters / Adam moments / EMA to --out; tests/test_gpu_dp.py compares
them (and the ranks among themselves).  Inputs of rank r at step k are drawn from a generator
seeded (1000 * k + r), identical in both modes.
"""
import argparse
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def inputs(rank, k, B):
    g = torch.Generator().manual_seed(1000 * (k + 2) + rank)
    img = torch.rand(B, 3, 64, 64, generator=g) * 2 - 1
    return img, torch.randint(0, 1000, (B,), generator=g), torch.randn(B, 3, 16, 16, generator=g)


def feed(f, rank, k, B):
    img, t, noise = inputs(rank, k, B)
    f["img"].copy_(img)
    f["t"].copy_(t)
    f["noise"].copy_(noise)


LR = 2e-4  # the DP job's lr = world * B * base_lr (main_val.py:834-838); the definition uses the same


def build(B, world):
    import encdiff_amd  # noqa: F401
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer
    torch.manual_seed(1234)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    ldm.use_scheduler = False  # constant lr: the updates carry the gradients
    tr = HipTrainer(ldm, B, base_lr=LR / (B * world), pool_size=4 * B)
    assert abs(tr.opt.param_groups[0]["lr"] - LR) < 1e-12
    return ldm, tr


def save(tr, path, extra):
    a = tr.arena
    h = hashlib.sha256()
    for buf in (a.master, a.exp_avg, a.exp_avg_sq):
        h.update(buf.detach().cpu().numpy().tobytes())
    torch.save({"master": a.master.cpu(), "exp_avg": a.exp_avg.cpu(), "exp_avg_sq": a.exp_avg_sq.cpu(),
                "ema": a.ema.cpu(), "digest": h.hexdigest(), **extra}, path)
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("dp", "w1"), required=True)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    B, W = args.batch, args.world
    if args.mode == "dp":
        import torch.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        dist.init_process_group("gloo")
        rank = dist.get_rank()
        ldm, tr = build(B, W)
        f = tr.enable_feed()
        feed(f, rank, -1, B)
        tr.init_scale_factor()  # rank 0's batch, broadcast
        grads, local = {}, {}
        for k in range(args.warmup):
            feed(f, rank, k, B)
            tr.buckets.record = {}
            tr.step_eager()
            grads[k] = tr.arena.grad.cpu().clone()  # the exchanged (averaged) gradient of step k
            rec = tr.buckets.record
            local[k] = torch.cat([rec[i] for i in sorted(rec)]).cpu()  # what this rank sent
            tr.buckets.record = None
        tr.capture(warmup=0)
        for k in range(args.warmup, args.warmup + args.steps):
            feed(f, rank, k, B)
            tr.step()
            grads[k] = tr.arena.grad.cpu().clone()
        torch.cuda.synchronize()
        d = save(tr, args.out + f".rank{rank}", dict(split_lo=tr._split_lo, loss=tr.loss(), grads=grads,
                                                        local=local))
        digests = [None] * W
        dist.all_gather_object(digests, d)
        if rank == 0:
            print(f"dp: split_lo={tr._split_lo} buckets={tr.buckets.bounds} ranks_equal={len(set(digests)) == 1}",
                  flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    # w1: the definition of the DP step on one process
    ldm, tr = build(B, 1)
    f = tr.enable_feed()
    a = tr.arena
    feed(f, 0, -1, B)
    tr.init_scale_factor()
    grads, local = {}, {}
    for k in range(args.warmup + args.steps):
        tr.opt.stage_hyper()
        acc = torch.zeros_like(a.grad)
        for r in range(W):
            feed(f, r, k, B)
            tr._fwd_bwd()   # zeroes the arena gradient, then UNet + Encoder4 backward
            local[(k, r)] = a.grad.cpu().clone()
            acc += a.grad
        a.grad.copy_(acc / W)  # the gloo exchange: sum over ranks, then / world
        grads[k] = a.grad.cpu().clone()
        tr.opt.launch()
        tr._post()
    torch.cuda.synchronize()
    save(tr, args.out, dict(grads=grads, local=local, names={n: a.offsets[n] for n in a.names}))
    print("w1: done", flush=True)


if __name__ == "__main__":
    main()

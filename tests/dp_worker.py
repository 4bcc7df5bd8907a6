"""One rank of the data-parallel GPU test (tests/test_gpu_dp.py): the product
DP path -- unet_amd.train.Trainer with a process group, its segmented
backward, the bucketed asynchronous all-reduce and the 1/world SGD scale --
on this rank's shard.  Ranks share the one GPU of the test box and talk over
gloo (RCCL needs one GPU per rank; the all-reduce call pattern is the same).

    python tests/dp_worker.py <out.npz> <overlap 0|1> <steps> [comm fp32|bf16] [precision fp32|bf16]
                              [batch] [size]
    env: RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT;
         UNET_DP_TUNE_DB=<path>: replay that GEMM tuning database (the bench's);
         UNET_DP_BACKEND=nccl: RCCL (one GPU per rank: world 1 on the test box),
         UNET_DP_FORCE=1: issue the collectives at world 1 too (Trainer force_collectives),
         UNET_DP_STEP=1: whole Trainer.step() calls (with the per-step buffer broadcast),
         UNET_DP_SYNC_BCAST=1: that broadcast synchronous ahead of every forward (not deferred),
         UNET_DP_RELOAD_AT=k: before step k every rank load_state_dict()s its model with new
           BatchNorm running statistics (UNET_DP_RELOAD_SYNC=1: then Trainer.sync_buffers()),
         UNET_DETERMINISTIC=1: the library's deterministic mode (no fp32 atomics)
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import fixtures as F  # noqa: E402  (test inputs only)
from oracle import unet_oracle as O  # noqa: E402

SEED, BATCH, SIZE = 51, 2, 188


def shard(rank, batch=BATCH, size=SIZE):
    return F.make_inputs(100 + rank, batch, 1, size)


def main():
    out, overlap, steps = sys.argv[1], bool(int(sys.argv[2])), int(sys.argv[3])
    comm = {"fp32": torch.float32, "bf16": torch.bfloat16}[sys.argv[4] if len(sys.argv) > 4 else "fp32"]
    precision = sys.argv[5] if len(sys.argv) > 5 else "fp32"
    batch = int(sys.argv[6]) if len(sys.argv) > 6 else BATCH
    size = int(sys.argv[7]) if len(sys.argv) > 7 else SIZE
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    backend = os.environ.get("UNET_DP_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    force = os.environ.get("UNET_DP_FORCE") == "1"
    from unet_amd import UNet, _lib
    from unet_amd.train import Trainer
    db = os.environ.get("UNET_DP_TUNE_DB")
    if db:
        n = _lib.load().unet_tuning_load(db.encode())
        assert n > 0, (db, n)
    params = O.hash_init(1, 2, seed=SEED, bn_random=True)
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.cuda().train()
    tr = Trainer(m, batch, size, size, lr=1e-4, momentum=0.99, process_group=dist.group.WORLD, overlap=overlap,
                 comm_dtype=comm, precision=precision, force_collectives=force)
    tr.defer_join = os.environ.get("UNET_DP_DEFER", "1") != "0"
    tr.defer_buffer_bcast = os.environ.get("UNET_DP_SYNC_BCAST") != "1"
    x, t, w = (torch.from_numpy(a).cuda() for a in shard(rank, batch, size))
    res = {}
    if os.environ.get("UNET_DP_STEP") == "1":
        starts = []
        tr.on_buffers_synced = lambda b: starts.append(b.double().cpu().numpy().copy())
        reload_at = int(os.environ.get("UNET_DP_RELOAD_AT", "-1"))
        _lib.load().unet_nondeterministic_sites(1)
        for s in range(steps):
            if s == reload_at:  # a checkpoint resume between steps, on every rank
                sd = {k: v.clone() for k, v in m.state_dict().items()}
                new = F.plausible_running_stats({k: v.cpu().numpy() for k, v in sd.items()}, 900 + s)
                m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in new.items()})
                res["reloaded"] = tr.flat_buffers.flat.double().cpu().numpy().copy()
                if os.environ.get("UNET_DP_RELOAD_SYNC") == "1":
                    tr.sync_buffers()
            res[f"loss{s}"] = np.array(tr.step(x, t, w).item())
            torch.cuda.synchronize()
            res[f"buf{s}"] = tr.flat_buffers.flat.double().cpu().numpy().copy()
        res["params"] = tr.flat.flat.cpu().numpy().copy()
        res["nondet_sites"] = np.array(_lib.load().unet_nondeterministic_sites(0))
        res["slab_fallbacks"] = np.array(_lib.slab_fallbacks())
        for s, b in enumerate(starts):
            res[f"start{s}"] = b  # the buffers each step's forward started from
        np.savez(out, **res)
        dist.barrier()
        dist.destroy_process_group()
        return
    for s in range(steps):
        res[f"w{s}"] = tr.flat.flat.cpu().numpy().copy()         # weights this step starts from
        loss = tr.forward_loss(x, t, w)
        tr.backward_and_reduce(x)
        torch.cuda.synchronize()
        res[f"grad{s}"] = tr.flat.grad.cpu().numpy().copy()     # SUM over ranks
        res[f"loss{s}"] = np.array(loss.item())
        tr.optimizer_step()
    torch.cuda.synchronize()
    res["params"] = tr.flat.flat.cpu().numpy().copy()
    res["backend"] = np.array(dist.get_backend())
    res["issued"] = np.array(tr.reducer.issued + tr.reducer_whole.issued)
    res["buffers_before_sync"] = np.concatenate([b.double().cpu().numpy().ravel() for b in m.buffers()])
    tr.sync_buffers()
    res["buffers"] = np.concatenate([b.double().cpu().numpy().ravel() for b in m.buffers()])
    if db:
        rep = _lib.tuning_report()
        res["tune_live"] = np.array(sum(1 for ln in rep.splitlines() if ln and "tuning db" not in ln))
    np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

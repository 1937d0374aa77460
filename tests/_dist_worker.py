"""Worker of the multi-process (gloo) tests: one rank of a world, MASTER at 127.0.0.1.

Runs llsr.dist.sharded_scan2map (the product driver) with the oracle's CPU engine for this rank's
share of the correspondences (gloo cannot drive the HIP kernels), plus the bench contract's
max-over-ranks timing, and reports through a multiprocessing queue."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for sub in ("lego-loam-sr_amd", "oracle"):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def run(rank, world, port, mode, iter_max, queries, q):
    try:
        import numpy as np
        import torch.distributed as dist
        import oracle_py
        from llsr import _abi
        from llsr.dist import max_over_ranks, shard_range, sharded_scan2map
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        z = np.load(os.path.join(HERE, "golden", "mo_map_vlp16.npz"))
        cfg = _abi.config_for("vlp16")
        cfg.mode = mode
        cfg.iterCountThres = iter_max
        probs = [(z[f"q{i}_corner"], z[f"q{i}_surf"], z["corner_map"], z["surf_map"], z[f"q{i}_init"])
                 for i in queries]
        eng = oracle_py.OracleShardEngine(cfg, probs)
        ne = eng.new_ne()
        iters = sharded_scan2map(eng, ne, cfg.iterCountThres)
        res = eng.results()
        t = max_over_ranks(0.001 * (rank + 1))
        q.put((rank, iters, [(r["pose"].tolist(), r["iterations"], r["converged"]) for r in res], t,
               list(shard_range(10, rank, world))))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure in the parent
        q.put((rank, "error", repr(e), None, None))

"""Child process of tests/test_gpu_rccl.py: a one-rank RCCL ("nccl") process group on cuda:0,
through which ShardedLogLik exchanges its partials exactly as N ranks do (the async
all_gather_into_tensor on the RCCL stream, the side-stream wait, combine_partials_out).
Exits 0 and prints RCCL_ONE_RANK_OK when every check holds."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import Covariance, ShardedLogLik  # noqa: E402
from pynngp_amd.sweep import PipelinedCombine, combine_partials  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    rng = np.random.default_rng(11)
    n, m = 200_000, 15
    c = torch.from_numpy(rng.uniform(0, 1, (n, 2))).to(dev)
    v = torch.from_numpy(rng.standard_normal(n)).to(dev)
    sw = ShardedLogLik(c, m, 0, 1, layout="storage")
    assert sw.collective, "a process group exists: the partials must go through the collective"
    covs = [Covariance("exponential", 1.0, phi, 0.0) for phi in (10.0, 20.0, 30.0, 45.0)]
    local = [sw.local_partials(cv, v).clone() for cv in covs]
    # the pipelined exchange (async all-gather + side-stream fold) equals the local partials bit for bit
    pipe = PipelinedCombine(sw, len(covs))
    assert pipe.active
    for k, cv in enumerate(covs):
        sw.local_partials(cv, v, False, out=pipe.local[k])
        pipe.exchange(k)
    res = pipe.finish()
    torch.cuda.synchronize()
    for k in range(len(covs)):
        assert torch.equal(res[k], local[k]), (k, res[k], local[k])
    # one all-gather per sweep, and 3 + 1 sweeps per all-gather (a partial last batch): the same bits
    for batch, n_coll in ((1, 4), (3, 2)):
        pipe = PipelinedCombine(sw, len(covs), batch=batch)
        for k, cv in enumerate(covs):
            sw.local_partials(cv, v, False, out=pipe.local[k])
            pipe.exchange(k)
        res = pipe.finish()
        torch.cuda.synchronize()
        assert pipe.n_collectives == n_coll
        for k in range(len(covs)):
            assert torch.equal(res[k], local[k]), (batch, k, res[k], local[k])
    # the blocking exchange too
    for k, cv in enumerate(covs):
        g = combine_partials(sw.local_partials(cv, v).clone(), 1, force=True)
        assert torch.equal(g, local[k])
    # loglik_scan (one host sync) equals one loglik call per covariance
    scan = sw.loglik_scan(covs, v)
    single = [sw.loglik(cv, v) for cv in covs]
    assert scan == single, (scan, single)
    # the same sweep without the collective gives the same numbers
    sw0 = ShardedLogLik(c, m, 0, 1, layout="storage", collective=False)
    assert [sw0.loglik(cv, v) for cv in covs] == single
    dist.destroy_process_group()
    print("RCCL_ONE_RANK_OK", single)


if __name__ == "__main__":
    main()

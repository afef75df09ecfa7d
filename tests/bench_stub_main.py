"""bench.py with its GPU workload replaced by a CPU stand-in, so the rank
logic the driver's multi-GPU runs depend on -- starting N ranks from
`bench.py --gpus N`, the world-size check, barriers and max-over-ranks
timing, the photon sum, the per-rank report gather, the parity / roofline
objects of the N>1 line -- runs on CPU with gloo (tests/test_bench_dist.py).
Test infrastructure only: the stand-in propagates nothing and the line it
prints is not a measurement.

STUB_FAIL_RANK=r makes rank r exit with status 3 after the process group is up;
STUB_PARITY_FAIL_RANK=r makes rank r's parity check fail.
"""
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class StubWorkload(object):
    def __init__(self, args, rank, world, local, dist, nphotons):
        if os.environ.get('STUB_FAIL_RANK') == str(rank):
            sys.exit(3)
        self.args, self.rank, self.world, self.nphotons = args, rank, world, nphotons
        self.dist = dist
        # the real setup path on the host: rank 0 fills the node-local cache (reference
        # BVH + traversal BVH), the other ranks load both from it
        from chroma.gpu import wide_bvh
        from chroma.gpu.packing import PackedGeometry
        self.det, self.setup = bench.shared_geometry(args.detector, args.cache_dir, rank, dist)
        t0 = time.time()
        self.setup['wide_bvh_source'] = wide_bvh.obtain(self.det.bvh, PackedGeometry(self.det))[1]
        self.setup['wide_bvh_s'] = round(time.time() - t0, 3)
        self.setup['host_threads'] = bench._native_host_threads()
        self.group = max(1, min(args.steps, args.pipeline_depth)) if args.pipeline else 1
        self.reduced = {}
        self.calls = []

    def sync(self):
        pass

    def run(self, m, pipeline=None):
        import torch
        from chroma.gpu import shard
        self.calls.append((m, self.args.pipeline if pipeline is None else pipeline))
        out = []
        for _ in range(m):
            time.sleep(0.01 * (self.rank + 1))
            counts = torch.zeros(4, dtype=torch.int32)
            counts[self.rank % 4] = 1 + self.rank
            self.reduced['counts'] = shard.allreduce_channel_counts(counts)
            out.append(SimpleNamespace(trace_ms=2.0 + self.rank, trace_launches=2, trace_rays=1000 * (self.rank + 1),
                                       trace_ms_n=2, trace_launch_ms=[1.0 + self.rank, 1.0],
                                       trace_launch_rays=[700 * (self.rank + 1), 300 * (self.rank + 1)],
                                       kernel_ms=3.0, launches=4, steps_run=3, host_syncs=1, stack_overflows=0,
                                       flat_walks=0, flat_walks_whole=0, tail_ms=0.5, tail_photons=10,
                                       tail_max_steps=5, tail_max_cycles=0, tail_slowest_steps=5,
                                       tail_long_photons=0, tail_long_ticks=0, tail_long_walk_ticks=0,
                                       tail_long_walk_iterations=0, tail_long_steps=0))
        return out

    def run_sequential(self, m):
        return self.run(m, pipeline=False)

    def rank_report(self, stats):
        return {'rank': self.rank, 'photons_per_step': self.nphotons, 'device': 'stub', 'local_rank': self.rank,
                'host': 'stub', 'kernel_ms': sum(s.kernel_ms for s in stats),
                'launches': sum(s.launches for s in stats), 'host_steps': sum(s.steps_run for s in stats),
                'host_syncs': sum(s.host_syncs for s in stats), 'trace_ms': sum(s.trace_ms for s in stats),
                'trace_launches': sum(s.trace_launches for s in stats),
                'trace_rays': sum(s.trace_rays for s in stats),
                'launch_ms': [x for s in stats for x in s.trace_launch_ms], 'launch_rays': [700, 300],
                'overflows': 0, 'flat': 0, 'flat_whole': 0, 'detected_last_step': 0,
                'channel_hits_all_ranks': int(self.reduced['counts'].sum().item()), 'tail': [],
                'setup': dict(self.setup, upload_s=0.0, setup_s=0.0, **bench.host_memory()),
                'calls': self.calls}

    def untimed_passes(self):
        return {}

    def device_info(self):
        return {'device': 'stub', 'kernels': []}

    def detector_info(self):
        return {'triangles': 0, 'bvh_nodes': 0, 'channels': 4}

    def _parity(self, rank, n, full, threads):
        ok = os.environ.get('STUB_PARITY_FAIL_RANK') != str(rank)
        return {'rank': rank, 'n': n, 'flags_equal': ok, 'last_hit_equal': True, 'channel_equal': True, 'ok': ok,
                'threads': threads, 'full': full, 'oracle_on_rank': self.rank,
                'rng_first_subsequence': bench.rng_first_subsequence(rank, self.args.nthreads_per_block *
                                                                     self.args.max_blocks)}

    def gpu_sample(self, n, pipeline):
        # what a rank > 0 sends to rank 0: its photons (here a stand-in array) and the run's facts
        import numpy as np
        return {'rank': self.rank, 'n': int(n), 'path': 'stub', 'stack_overflows': 0,
                'photons': {'flags': np.full(n, self.rank, np.uint32)}}

    def check(self, full, budget_s, threads, sample):
        stats = {'nodes_visited': 1000, 'tris_tested': 100, 'traversals': 10}
        cpu = {'value': 1.0, 'unit': 'photons/s', 'cores': threads, 'kind': 'port', 'sample': 'stub'} if full else None
        return cpu, stats, self._parity(self.rank, 100 if full else min(self.nphotons, sample), full, threads)

    def check_rank(self, sample, threads):
        # rank 0 checks another rank's sample: the sample must be that rank's own
        assert self.rank == 0 and (sample['photons']['flags'] == sample['rank']).all()
        return self._parity(sample['rank'], sample['n'], False, threads)


bench.WORKLOAD = StubWorkload

if __name__ == '__main__':
    sys.exit(bench.main())

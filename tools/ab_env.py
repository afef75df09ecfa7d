#!/usr/bin/env python
"""In-process A/B of library switches that are read per launch (CHR_* env
variables): one geometry build + upload, then every configuration propagates
the bench workload (bench.PropagateWorkload) in interleaved rounds, so box and
thermal drift hit all configurations alike.  Per configuration and round: the
pipelined photons/s over the timed steps and the trace / tail diagnostics; and
once per configuration, the photons of one propagate from a re-initialised
RNG, hashed: every configuration must give the same photons (they are A/B
switches, not different physics).  Dev tool (GPU box).

usage: tools/ab_env.py [bench args] -- NAME=ENV:V,ENV:V  NAME2=...  (NAME=: the defaults)
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    split = argv.index('--')
    bench_args, configs = argv[:split], argv[split + 1:]
    rounds = int(os.environ.get('AB_ROUNDS', '2'))
    import bench
    import torch
    args = bench.parse_args(bench_args)
    torch.cuda.set_device(0)
    wl = bench.WORKLOAD(args, 0, 1, 0, None, args.photons)
    from chroma import gpu
    parsed = []
    for c in configs:
        name, _, rest = c.partition('=')
        env = dict(kv.split(':', 1) for kv in rest.split(',') if kv)
        parsed.append((name, env))
    base_env = {k: os.environ.get(k) for _, env in parsed for k in env}

    def apply(env):
        for k, v in base_env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        os.environ.update(env)

    hashes = {}
    for name, env in parsed:       # identical photons under every switch
        apply(env)
        wl.rng = gpu.get_rng_states(wl.nslots, seed=args.seed)
        wl.run(1)
        gp = wl.reduced.pop('gp')
        h = hashlib.sha256()
        for f in ('flags', 'last_hit_triangles', 'pos', 't'):
            h.update(getattr(gp, f).get().tobytes())
        hashes[name] = h.hexdigest()[:16]
        print(json.dumps({'config': name, 'env': env, 'photons_sha': hashes[name]}), flush=True)
    same = len(set(hashes.values())) == 1
    print(json.dumps({'photons_identical_across_configs': same}), flush=True)
    for r in range(rounds):
        for name, env in parsed:
            apply(env)
            # the same RNG start for every configuration: identical batches, tails and walks
            wl.rng = gpu.get_rng_states(wl.nslots, seed=args.seed)
            elapsed, per_step, stats = bench.timed_loop(wl.run, args.steps, max(2, args.warmup), None, wl.sync,
                                                        wl.group)
            rep = wl.rank_report(stats)
            wl.reduced.pop('gp', None)
            tails = [t for t in rep['tail'] if t['long_photons']]
            print(json.dumps({
                'config': name, 'round': r, 'photons_per_s': args.photons * args.steps / elapsed,
                'ms_per_step': 1e3 * elapsed / args.steps,
                'trace_ms_per_step': rep['trace_ms'] / args.steps,
                'kernel_ms_per_step': rep['kernel_ms'] / args.steps,
                # tail launch times need CHR_SLOT_TIMING=1; otherwise the slowest photon's time
                'tail_ms_mean': sum(t['ms'] or t['slowest_photon_ms'] for t in rep['tail']) / max(1, len(rep['tail'])),
                'long_us_per_step': [t['long_us_per_step'] for t in tails],
                'long_walk_us_per_step': [t['long_walk_us_per_step'] for t in tails],
                'first_trace_launches_ms': [round(x, 3) for x in rep['launch_ms'][:10]],
                'time': time.time()}), flush=True)
    return 0 if same else 1


if __name__ == '__main__':
    sys.exit(main())

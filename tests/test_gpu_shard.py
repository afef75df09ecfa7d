"""Photon-sharded Simulation (chroma.sim.ShardedSimulation) with two ranks on
the one GPU of the test box (gloo carries the collectives; production runs
use RCCL on one GPU per rank).  Each rank's propagation, the gathered hits and
the reduced DAQ channels are checked against the CPU oracle run on the same
slices with the same RNG subsequences."""
import os
import socket
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NTPB, MAXB, NEV, PER_EV = 256, 256, 4, 5000      # S = 65,536 slots; 20,000 photons -> one launch per rank


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _detector():
    from chroma import demo, loader
    det = loader.create_geometry_from_obj(demo.detector(600.0, 900.0, 1500.0))
    det.set_time_dist_gaussian(1.2, -6.0, 6.0)
    det.set_charge_dist_gaussian(1.0, 0.1, 0.5, 1.5)
    return det


def _photons():
    from chroma.photon_source import isotropic
    return isotropic(NEV * PER_EV, seed=41)


def _worker(rank, world, port, out_dir, hits):
    sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))
    os.environ['LOCAL_RANK'] = '0'        # both ranks drive the box's one GPU
    import torch.distributed as dist
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        from chroma.sim import ShardedSimulation
        sim = ShardedSimulation(_detector(), seed=1, nthreads_per_block=NTPB, max_blocks=MAXB, hits=hits)
        ph = _photons()
        evs = list(sim.simulate([ph[i * PER_EV:(i + 1) * PER_EV] for i in range(NEV)], run_daq=True,
                                keep_hits=False))
        out = {}
        for i, ev in enumerate(evs):
            h = ev.flat_hits
            if h is None:          # hits='root': only rank 0 receives the gathered hits
                assert rank != 0 and hits == 'root'
                out['ch_t_%d' % i] = ev.channels.t
                out['ch_q_%d' % i] = ev.channels.q
                out['ch_flags_%d' % i] = ev.channels.flags
                continue
            out['flags_%d' % i] = h.flags
            out['last_hit_%d' % i] = h.last_hit_triangles
            out['channel_%d' % i] = h.channel
            out['pos_%d' % i] = h.pos
            out['t_%d' % i] = h.t
            out['ch_t_%d' % i] = ev.channels.t
            out['ch_q_%d' % i] = ev.channels.q
            out['ch_flags_%d' % i] = ev.channels.flags
        np.savez(os.path.join(out_dir, 'rank%d.npz' % rank), **out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('hits', ['root', 'all'])
def test_sharded_simulation_two_ranks(tmp_path, hits):
    """DAQ on: one propagate per batch (the DAQ draws from rng_states between
    batches).  hits='root' gathers the hits to rank 0 only, 'all' to both."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), hits), nprocs=2, join=True)
    got = [np.load(os.path.join(str(tmp_path), 'rank%d.npz' % r)) for r in range(2)]
    for k in got[1].files:                       # every rank yields the same events (hits: where gathered)
        assert np.array_equal(got[0][k], got[1][k]), k
    assert ('flags_0' in got[1].files) == (hits == 'all')

    from chroma.gpu.detector import cdf_arrays
    from chroma.gpu.packing import PackedGeometry
    det = _detector()
    packed = PackedGeometry(det)
    ph = _photons()
    n = len(ph)
    S = NTPB * MAXB
    unit = np.float32(det.charge_cdf[0][-1] / 2 ** 16)
    hits_idx, hits_ch, hosts, daq_words = [], [], [], []
    for r in range(2):
        lo, hi = n * r // 2, n * (r + 1) // 2
        host = oracle.HostPhotons(ph[lo:hi])
        host.flags[:] = 0
        host.last_hit_triangles[:] = -1
        host.weights[:] = 1
        st = oracle.rng_init(S, seed=1, first_subsequence=r * S)
        oracle.propagate(packed, host, st, S, NTPB, MAXB, 1000)
        idx, ch = oracle.hits(host, det.solid_id, det.solid_id_to_channel_index)
        hits_idx.append(idx + lo)
        hits_ch.append(ch)
        hosts.append((lo, hi, host))
        words = []
        for e in range(NEV):
            a, b = max(e * PER_EV, lo), min((e + 1) * PER_EV, hi)
            words.append(oracle.daq(host, det.solid_id, det.solid_id_to_channel_index, cdf_arrays(det.time_cdf),
                                    cdf_arrays(det.charge_cdf), unit, st, S, start=a - lo, n=max(0, b - a),
                                    nchannels=det.num_channels(), nthreads_per_block=NTPB, max_blocks=MAXB,
                                    raw=True))
        daq_words.append(words)
    gidx = np.concatenate(hits_idx)
    gch = np.concatenate(hits_ch)

    def host_field(f, i):
        for lo, hi, h in hosts:
            if lo <= i < hi:
                return getattr(h, f)[i - lo]
    for e in range(NEV):
        sel = (gidx >= e * PER_EV) & (gidx < (e + 1) * PER_EV)
        idx = gidx[sel]
        assert np.array_equal(got[0]['channel_%d' % e], gch[sel])
        assert np.array_equal(got[0]['flags_%d' % e], np.array([host_field('flags', i) for i in idx], np.uint32))
        assert np.array_equal(got[0]['last_hit_%d' % e], np.array([host_field('last_hit_triangles', i) for i in idx]))
        assert np.allclose(got[0]['pos_%d' % e], np.array([host_field('pos', i) for i in idx]).reshape(-1, 3),
                           rtol=1e-5, atol=1e-5)
        t = np.minimum(daq_words[0][e][0], daq_words[1][e][0])
        q = (daq_words[0][e][1].astype(np.uint64) + daq_words[1][e][1]).astype(np.uint32)
        fl = daq_words[0][e][2] | daq_words[1][e][2]
        assert np.array_equal(got[0]['ch_t_%d' % e].view(np.uint32), t)
        assert np.array_equal(got[0]['ch_q_%d' % e], (q.astype(np.float32) * unit).astype(np.float32))
        assert np.array_equal(got[0]['ch_flags_%d' % e], fl)
    assert len(gidx) > 100


SIZES = (5000, 1, 4000, 3000)   # photons_per_batch=1: one batch per event; the 1-photon batch leaves rank 0 empty


def _pipe_worker(rank, world, port, out_dir, hits):
    sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))
    os.environ['LOCAL_RANK'] = '0'
    import torch.distributed as dist
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        from chroma.photon_source import isotropic
        from chroma.sim import ShardedSimulation
        ph = isotropic(sum(SIZES), seed=43)
        cuts = np.cumsum((0,) + SIZES)
        out = {}
        for depth in (8, 1):
            sim = ShardedSimulation(_detector(), seed=5, nthreads_per_block=NTPB, max_blocks=MAXB, hits=hits)
            sim.pipeline_batches = depth
            evs = list(sim.simulate([ph[cuts[i]:cuts[i + 1]] for i in range(len(SIZES))], run_daq=False,
                                    keep_hits=False, photons_per_batch=1, keep_photons_end=True))
            out['pipeline_%d' % depth] = np.array(sim.last_pipeline)
            for i, ev in enumerate(evs):
                if ev.flat_hits is None:
                    assert rank != 0 and hits == 'root' and ev.photons_end is None
                    continue
                for f in ('flags', 'last_hit_triangles', 'channel', 't'):
                    out['%s_%d_%d' % (f, depth, i)] = getattr(ev.flat_hits, f)
                out['pos_%d_%d' % (depth, i)] = ev.flat_hits.pos
                # the end photons, gathered in global photon order
                for f in ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'last_hit_triangles', 'weights', 'evidx'):
                    out['end_%s_%d_%d' % (f, depth, i)] = getattr(ev.photons_end, f)
        np.savez(os.path.join(out_dir, 'rank%d.npz' % rank), **out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('hits', ['root', 'all'])
def test_sharded_simulation_pipelined(tmp_path, hits):
    """DAQ off: each rank propagates its shards of all batches in ONE pipelined
    propagate_batches call (empty shards left out of it: rank 0 holds nothing of
    the 1-photon batch), then the hits and the end photons of every batch are
    gathered in batch order.  The events equal the depth-1 run's (one propagate
    per batch), and the end photons equal the oracle's."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import torch.multiprocessing as mp
    mp.spawn(_pipe_worker, args=(2, _free_port(), str(tmp_path), hits), nprocs=2, join=True)
    got = [np.load(os.path.join(str(tmp_path), 'rank%d.npz' % r)) for r in range(2)]
    for g in got:
        assert tuple(g['pipeline_8']) == (len(SIZES), 1) and tuple(g['pipeline_1']) == (len(SIZES), 0)
    ranks_with_hits = (0, 1) if hits == 'all' else (0,)
    nhits = 0
    for r in ranks_with_hits:
        for i in range(len(SIZES)):
            for f in ('flags', 'last_hit_triangles', 'channel', 't', 'pos'):
                a, b = got[r]['%s_8_%d' % (f, i)], got[r]['%s_1_%d' % (f, i)]
                assert np.array_equal(a, b), (r, i, f)
                assert np.array_equal(a, got[0]['%s_8_%d' % (f, i)]), (r, i, f)
            nhits += len(got[r]['flags_8_%d' % i])
    if hits == 'root':
        assert 'flags_8_0' not in got[1].files and 'end_flags_8_0' not in got[1].files
    assert nhits > 50

    # keep_photons_end: each event's end photons == the oracle's for every rank's
    # slice of each batch, in global photon order (rank r: RNG subsequences from
    # r*S, one state set carried across the batches; empty shards not propagated)
    from chroma.gpu.packing import PackedGeometry
    from chroma.photon_source import isotropic
    packed = PackedGeometry(_detector())
    ph = isotropic(sum(SIZES), seed=43)
    cuts = np.cumsum((0,) + SIZES)
    S = NTPB * MAXB
    states = [oracle.rng_init(S, seed=5, first_subsequence=r * S) for r in range(2)]
    for i, n in enumerate(SIZES):
        parts = []
        for r in range(2):
            lo, hi = n * r // 2, n * (r + 1) // 2
            host = oracle.HostPhotons(ph[cuts[i] + lo:cuts[i] + hi])
            host.flags[:] = 0
            host.last_hit_triangles[:] = -1
            host.weights[:] = 1
            if hi > lo:
                oracle.propagate(packed, host, states[r], S, NTPB, MAXB, 1000)
            parts.append(host)
        for r in ranks_with_hits:
            for depth in (8, 1):
                for f in ('flags', 'last_hit_triangles'):
                    exp = np.concatenate([getattr(h, f) for h in parts])
                    assert np.array_equal(got[r]['end_%s_%d_%d' % (f, depth, i)], exp), (r, depth, i, f)
                for f in ('pos', 'dir', 'pol', 't', 'wavelengths'):
                    exp = np.concatenate([np.asarray(getattr(h, f)) for h in parts]).reshape(n, -1)
                    g = got[r]['end_%s_%d_%d' % (f, depth, i)].reshape(n, -1)
                    assert np.allclose(g, exp, rtol=1e-5, atol=1e-5), (r, depth, i, f)
                assert (got[r]['end_evidx_%d_%d' % (depth, i)] == 0).all()

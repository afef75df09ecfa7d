"""Simulation.simulate with pipelined batches: closed
batches are read ahead from the iterable and propagated by one
chr_propagate_batches call (batch k's tail on a second stream under batch
k+1's first step).  The contract is the reference's one-batch-at-a-time loop
(sim.py:112-160, _simulate_batch sim.py:54-110): same batches (events never
split), same per-event evidx, hits and photons, same RNG slot states after --
checked against the sequential oracle and against pipeline_batches = 1.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

SIZES = (6000, 9000, 3000, 12000, 5000, 8000, 4000)
PER_BATCH = 10000          # batches: [6k, 9k] [3k, 12k] [5k, 8k] [4k]
NTPB, MAXB, STEPS, SEED = 64, 128, 1000, 7


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    torch.cuda.set_device(0)


def _events():
    from chroma.photon_source import isotropic
    return [isotropic(n, seed=100 + i) for i, n in enumerate(SIZES)]


def _batches():
    out, cur, n = [], [], 0
    for i, s in enumerate(SIZES):
        cur.append(i)
        n += s
        if n >= PER_BATCH:
            out.append(cur)
            cur, n = [], 0
    if cur:
        out.append(cur)
    return out


def _oracle(det, packed):
    """The reference's loop on the CPU: each batch joined, evidx = event index
    inside the batch, propagated in order with one set of RNG slot states."""
    from chroma.event import Photons
    evs = _events()
    nslots = NTPB * MAXB
    states = oracle.rng_init(nslots, seed=SEED)
    per_event = {}
    for batch in _batches():
        joined = Photons.join([evs[i] for i in batch])
        joined.evidx[:] = np.repeat(np.arange(len(batch)), [SIZES[i] for i in batch])
        host = oracle.HostPhotons(joined)
        host.last_hit_triangles[:] = -1
        host.weights[:] = 1.0
        oracle.propagate(packed, host, states, nslots, NTPB, MAXB, STEPS)
        idx, ch = oracle.hits(host, det.solid_id, det.solid_id_to_channel_index)
        off = 0
        for k, i in enumerate(batch):
            sl = slice(off, off + SIZES[i])
            sel = (idx >= off) & (idx < off + SIZES[i])
            per_event[i] = dict(flags=host.flags[sl].copy(), last_hit=host.last_hit_triangles[sl].copy(),
                                pos=host.pos[sl].copy(), t=host.t[sl].copy(), hit_idx=idx[sel] - off,
                                hit_ch=ch[sel], evidx=k)
            off += SIZES[i]
    return per_event, states


def _simulate(det, depth):
    from chroma.sim import Simulation
    sim = Simulation(det, seed=SEED, nthreads_per_block=NTPB, max_blocks=MAXB)
    sim.pipeline_batches = depth
    out = list(sim.simulate(_events(), keep_photons_end=True, max_steps=STEPS, photons_per_batch=PER_BATCH))
    return out, sim.rng_states.get(), sim.last_pipeline


@pytest.mark.parametrize('depth', [8, 3, 1])
def test_simulate_pipelined_equals_sequential_oracle(cuda, small_detector, small_packed, depth):
    ref, states = _oracle(small_detector, small_packed)
    out, rng, (nbatches, calls) = _simulate(small_detector, depth)
    assert nbatches == len(_batches()) == 4
    assert calls == {8: 1, 3: 1, 1: 0}[depth]      # pipelined calls: [4] / [3 + 1 single] / none
    assert len(out) == len(SIZES)
    for i, ev in enumerate(out):
        r = ref[i]
        pe = ev.photons_end
        assert np.array_equal(pe.flags, r['flags']), 'event %d flags' % i
        assert np.array_equal(pe.last_hit_triangles, r['last_hit']), 'event %d last hit' % i
        assert np.allclose(pe.pos, r['pos'], rtol=1e-5, atol=1e-5)
        assert np.allclose(pe.t, r['t'], rtol=1e-5, atol=1e-6)
        fh = ev.flat_hits
        assert np.array_equal(fh.channel.astype(np.int64), r['hit_ch'].astype(np.int64)), 'event %d channels' % i
        assert np.array_equal(fh.flags, r['flags'][r['hit_idx']])
        assert (fh.evidx == r['evidx']).all()
        assert sum(len(v) for v in ev.hits.values()) == len(fh)
    assert np.array_equal(rng.reshape(-1), states.reshape(-1))


def test_simulate_with_daq_stays_sequential(cuda):
    """run_daq=True: the DAQ draws from rng_states between batches, so
    simulate() keeps one propagate per batch (no pipelined call)."""
    from chroma import demo, loader
    from chroma.sim import Simulation
    det = loader.create_geometry_from_obj(demo.detector(600.0, 900.0, 1500.0))
    det.set_time_dist_gaussian(1.2, -6.0, 6.0)
    det.set_charge_dist_gaussian(1.0, 0.1, 0.5, 1.5)
    sim = Simulation(det, seed=SEED, nthreads_per_block=NTPB, max_blocks=MAXB)
    out = list(sim.simulate(_events()[:4], run_daq=True, max_steps=STEPS, photons_per_batch=PER_BATCH))
    assert len(out) == 4 and all(ev.channels is not None for ev in out)
    assert sim.last_pipeline == (2, 0)

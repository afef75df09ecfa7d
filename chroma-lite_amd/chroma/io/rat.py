"""The RAT <-> Chroma ZeroMQ wire format (reference bin/chroma-server-rat:29-70).

Request (RAT -> Chroma), little-endian:
    u32 numphotons, u32 eventid
    11 f64 planes of numphotons values: x y z dx dy dz polx poly polz wavelength t
    u32 trackid[numphotons]
Reply (Chroma -> RAT):
    u32 nhits, u32 eventid
    11 f32 planes of nhits values (the hit photons' fields, float32 as the
    propagator holds them), hits grouped by channel in ascending channel order
    and, within a channel, in photon order (sim.py:137 builds the per-channel
    dict from np.unique)
    u32 channel[nhits] (the reference's stand-in for track ids), u32 channel[nhits]

Difference: the reference slices the track ids from byte 8*11*n instead of
8 + 8*11*n (it keeps the last 8 bytes of the t plane and drops the last two
ids); the ids are unused there.  decode_request reads them at their offset.
"""
import sys

import numpy as np

from chroma import event

PLANES = ('x', 'y', 'z', 'dx', 'dy', 'dz', 'polx', 'poly', 'polz', 'wavelength', 't')


def encode_request(photons, eventid, trackids=None):
    n = len(photons)
    trackids = np.zeros(n, dtype=np.uint32) if trackids is None else np.asarray(trackids, dtype=np.uint32)
    if len(trackids) != n:
        raise ValueError('one track id per photon')
    planes = np.concatenate([photons.pos.T, photons.dir.T, photons.pol.T, photons.wavelengths[None, :],
                             photons.t[None, :]]).astype('<f8')
    return np.asarray([n, eventid], dtype='<u4').tobytes() + planes.tobytes() + trackids.astype('<u4').tobytes()


def decode_request(msg):
    """-> (event.Photons, eventid, trackids)"""
    msg = memoryview(msg)
    if len(msg) < 8:
        raise ValueError('RAT request shorter than its header')
    n, eventid = (int(v) for v in np.frombuffer(msg[:8], dtype='<u4'))
    need = 8 + 8 * 11 * n
    if len(msg) < need:
        raise ValueError('RAT request of %d bytes for %d photons (expected at least %d)' % (len(msg), n, need))
    planes = np.frombuffer(msg[8:need], dtype='<f8').reshape(11, n)
    # the track-id block is optional: the reference server slices it loosely
    # (bin/chroma-server-rat:34) and never uses it
    tail = msg[need:]
    trackids = np.frombuffer(tail[:len(tail) - len(tail) % 4], dtype='<u4').copy()
    photons = event.Photons(planes[0:3].T, planes[3:6].T, planes[6:9].T, planes[9], planes[10])
    return photons, eventid, trackids


def encode_reply(hits, eventid):
    """hits: {channel: event.Photons} (Simulation keep_hits=True)."""
    chans = sorted(int(c) for c in hits)
    parts = [hits[c] for c in chans]
    n = sum(len(p) for p in parts)
    chanidx = np.concatenate([np.full(len(p), c, dtype='<u4') for c, p in zip(chans, parts)]) if parts \
        else np.zeros(0, dtype='<u4')

    def plane(get):
        return np.concatenate([get(p) for p in parts]).astype('<f4').tobytes() if parts else b''
    out = np.asarray([n, eventid], dtype='<u4').tobytes()
    for axis in range(3):
        out += plane(lambda p: p.pos[:, axis])
    for axis in range(3):
        out += plane(lambda p: p.dir[:, axis])
    for axis in range(3):
        out += plane(lambda p: p.pol[:, axis])
    out += plane(lambda p: p.wavelengths)
    out += plane(lambda p: p.t)
    return out + chanidx.tobytes() + chanidx.tobytes()


def decode_reply(msg):
    """-> (event.Photons with .channel, eventid)"""
    msg = memoryview(msg)
    n, eventid = (int(v) for v in np.frombuffer(msg[:8], dtype='<u4'))
    need = 8 + 4 * 11 * n + 8 * n
    if len(msg) != need:
        raise ValueError('RAT reply of %d bytes for %d hits (expected %d)' % (len(msg), n, need))
    planes = np.frombuffer(msg[8:8 + 44 * n], dtype='<f4').reshape(11, n)
    chans = np.frombuffer(msg[8 + 44 * n + 4 * n:], dtype='<u4')
    p = event.Photons(planes[0:3].T, planes[3:6].T, planes[6:9].T, planes[9], planes[10])
    p.channel = chans.copy()
    return p, eventid


def handle_request(sim, msg, max_steps=1000):
    """One request of chroma-server-rat: propagate the photons as one event
    (no DAQ: RAT digitises) and build the reply from the per-channel hits."""
    photons, eventid, _ = decode_request(msg)
    ev = next(sim.simulate(photons, keep_photons_beg=False, keep_photons_end=False, keep_hits=True,
                           run_daq=False, max_steps=max_steps))
    return encode_reply(ev.hits, eventid)


def serve(detector, address='ipc:///tmp/ipc_chroma', max_requests=None):
    """The chroma-server-rat loop (ZeroMQ REP socket).  Needs pyzmq."""
    try:
        import zmq
    except ImportError as e:
        raise ImportError('chroma-server-rat needs pyzmq (not installed in this environment)') from e
    from chroma.sim import Simulation
    from chroma.loader import load_geometry_from_string
    geo = load_geometry_from_string(detector) if isinstance(detector, str) else detector
    sim = Simulation(geo)
    socket = zmq.Context().socket(zmq.REP)
    socket.bind(address)
    served = 0
    while max_requests is None or served < max_requests:
        msg = socket.recv()
        try:
            reply = handle_request(sim, msg)
        except ValueError as e:       # malformed request: empty reply keeps the REP state machine going
            print('chroma-server-rat: bad request: %s' % e, file=sys.stderr, flush=True)
            eventid = int(np.frombuffer(msg[4:8], dtype='<u4')[0]) if len(msg) >= 8 else 0
            reply = encode_reply({}, eventid)
        socket.send(reply)
        served += 1

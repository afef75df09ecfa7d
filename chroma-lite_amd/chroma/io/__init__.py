"""Photon I/O formats either side of the propagator:
the RAT ZeroMQ wire format of bin/chroma-server-rat (chroma.io.rat) and the
photon archives of bin/chroma-profile --photons-npz (chroma.io.photons_npz).
The reference's ROOT writer (chroma/io/root.py) needs ROOT and is out of
scope."""

"""Log-frame parity helper for the GPU tests: the engine's zb_serialize_frames output must equal the oracle's
frames (oracle/zbref.cpp encode_frame) byte for byte. On a mismatch the first differing frame is reported
field by field."""
from zeebe_amd import records as R

FRAME_CFG = dict(stream_id=3, raft_term=2, timestamp=1_700_000_000_123)


def assert_frames_equal(o, e, start=0):
    fo = o.frames(start, -1, **FRAME_CFG)
    fe = e.frames(start, None, **FRAME_CFG)
    if fo == fe:
        return
    a, b = R.parse_frames(fo), R.parse_frames(fe)
    assert len(a) == len(b), ("frame count", len(a), len(b))
    for x, y in zip(a, b):
        if x != y:
            diff = {k: (x[k], y[k]) for k in x if x[k] != y[k]}
            raise AssertionError("frame at position %d differs: %s" % (x["position"], diff))
    raise AssertionError("frame bytes differ (padding)")

"""TP control plane (llmctl.serve.control): packed plan records and the shm / gloo channels."""

import numpy as np
import pytest
import torch

from llmctl.serve.control import pack, unpack
from llmctl.testing.harness import run_ranks
from llmctl.testing.workers import control_channel_worker


def test_pack_roundtrip_generic_and_decode():
    pre = {"op": "prefill", "ids": np.arange(9, dtype=np.int64), "pos": np.arange(9, dtype=np.int32),
           "bt": np.ones((2, 3), dtype=np.int32), "cu": [0, 4, 9], "doc": None, "x": 2.5, "ok": False, "n": -3,
           "name": "abc"}
    got = unpack(pack({"op": "mixed", "prefill": pre, "decode": {"op": "decode", "ids": [1, 2]}}))
    p = got["prefill"]
    assert got["op"] == "mixed" and got["decode"] == {"op": "decode", "ids": [1, 2]}
    assert p["cu"] == [0, 4, 9] and p["doc"] is None and p["x"] == 2.5 and p["ok"] is False and p["n"] == -3
    assert p["name"] == "abc" and p["pos"].dtype == np.int32 and (p["bt"] == 1).all() and p["bt"].shape == (2, 3)
    dec = {"op": "decode", "ids": [5, 6, 7], "positions": [1, 2, 3], "slots": [9, 8, 7], "ctx": [2, 3, 4],
           "bt": np.arange(6, dtype=np.int32).reshape(3, 2)}
    d = unpack(pack(dec))  # fixed-layout fast path
    assert d.keys() == dec.keys() and all((np.asarray(d[k]) == np.asarray(dec[k])).all() for k in dec if k != "op")


@pytest.mark.parametrize("kind,slot", [("shm", 8 << 20), ("shm", 4096), ("tensor", 0)])
def test_control_channel_multirank(kind, slot):
    out = run_ranks(control_channel_worker, 3, kind, slot)
    for r in (1, 2):
        assert torch.equal(out[r]["digest"], out[0]["digest"])
    if kind == "shm" and slot == 4096:
        assert int(out[0]["spilled"]) > 0  # big prefill plans went through the gloo fallback


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("victim,mode", [(0, "kill"), (2, "kill"), (0, "stop")])
def test_shm_channel_peer_loss(victim, mode):
    """A dead (or frozen) rank 0 / a dead reader: every survivor raises PeerLostError and exits
    non-zero within the deadline (2 s heartbeat deadline here) instead of spinning forever, and no
    /dev/shm ring file is left behind."""
    import glob
    import os
    import signal
    import subprocess
    import sys
    import time

    before = set(glob.glob("/dev/shm/llmctl-tp-*"))
    port, world = _free_port(), 3
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, "-m", "llmctl.testing.shm_liveness", "--rank", str(r), "--world",
                               str(world), "--port", str(port), "--victim", str(victim), "--mode", mode],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
             for r in range(world)]
    t0 = time.monotonic()
    try:
        survivors = [p for r, p in enumerate(procs) if r != victim]
        for p in survivors:
            p.wait(timeout=90)
        elapsed = time.monotonic() - t0
        logs = [p.stdout.read() for p in survivors]
        for p, log in zip(survivors, logs):
            assert p.returncode == 3, log
            assert "PeerLostError" in log, log
        assert elapsed < 60, elapsed  # setup (~imports) + detection, not an unbounded spin
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGKILL)
                p.wait(timeout=30)
    if mode == "kill":
        assert procs[victim].returncode == -signal.SIGKILL
    assert set(glob.glob("/dev/shm/llmctl-tp-*")) <= before


def test_pack_roundtrip_property():
    """Property test (hypothesis): any plan of the supported value kinds -- None / bool / int /
    float / str / int lists / numpy arrays of any shape and int / bool / float dtype / nested
    dicts, plus the fixed-layout decode and sampling-decode records -- survives pack -> unpack."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    from hypothesis.extra import numpy as hnp

    dtypes = st.sampled_from([np.int32, np.int64, np.float32, np.float64, np.bool_, np.uint8])
    arrays = dtypes.flatmap(lambda dt: hnp.arrays(dt, hnp.array_shapes(min_dims=0, max_dims=3, max_side=5)))
    leaves = st.one_of(st.none(), st.booleans(), st.integers(-2**62, 2**62), st.floats(allow_nan=False),
                       st.text(max_size=12), st.lists(st.integers(-2**31, 2**31), max_size=6), arrays)
    keys = st.text(alphabet="abcdefghij_", min_size=1, max_size=6)
    plans = st.recursive(st.dictionaries(keys, leaves, max_size=5),
                         lambda inner: st.dictionaries(keys, st.one_of(leaves, inner), max_size=4), max_leaves=12)

    def same(a, b):
        if isinstance(a, dict):
            return isinstance(b, dict) and a.keys() == b.keys() and all(same(a[k], b[k]) for k in a)
        if isinstance(a, np.ndarray):
            return (isinstance(b, np.ndarray) and a.dtype == b.dtype and a.shape == b.shape
                    and np.ascontiguousarray(a).tobytes() == b.tobytes())  # bitwise (NaN payloads too)
        if isinstance(a, list):
            return list(b) == a
        return type(a) is type(b) and a == b

    @settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
    @given(plans)
    def generic(plan):
        plan = dict(plan, op="prefill")
        assert same(plan, unpack(pack(plan)))

    @settings(max_examples=60, deadline=None)
    @given(st.integers(1, 17), st.integers(1, 9), st.booleans(), st.booleans())
    def decode(n, mb, sampling, cont):
        rng = np.random.default_rng(n * 31 + mb)
        plan = {"op": "decode_s" if sampling else "decode", "ids": rng.integers(0, 32000, n).tolist(),
                "positions": rng.integers(0, 4096, n).tolist(), "slots": rng.integers(-1, 1 << 20, n).tolist(),
                "ctx": rng.integers(1, 4096, n).tolist(), "bt": rng.integers(0, 999, (n, mb)).astype(np.int32)}
        if sampling:
            plan.update(cont=cont, u=rng.random(n, dtype=np.float32), temp=rng.random(n, dtype=np.float32),
                        topk=rng.integers(0, 50, n).astype(np.int32), topp=rng.random(n, dtype=np.float32))
        got = unpack(pack(plan))
        assert got["op"] == plan["op"]
        for k in ("ids", "positions", "slots", "ctx"):
            assert np.array_equal(got[k], np.asarray(plan[k]))
        assert np.array_equal(got["bt"], plan["bt"])
        if sampling:
            assert got["cont"] == cont
            for k in ("u", "temp", "topk", "topp"):
                assert np.array_equal(got[k], plan[k])

    generic()
    decode()

"""Child process for the shm control-plane liveness tests (tests/serve/test_control.py).

    python -m llmctl.testing.shm_liveness --rank R --world W --port P --victim V --mode kill|stop

Rank 0 publishes decode plans, the other ranks receive them.  The victim rank stops part-way:
``kill`` = SIGKILL itself (a crashed rank), ``stop`` = SIGSTOP itself (a frozen rank; the test
kills it afterwards).  Every survivor must leave with exit code 3 (``PeerLostError``) within the
channel's deadline instead of spinning forever; 0 would mean it never noticed.
"""

from __future__ import annotations

import argparse
import os
import signal
import sys
import time


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--victim", type=int, required=True)
    ap.add_argument("--mode", default="kill", choices=["kill", "stop"])
    ap.add_argument("--timeout", type=float, default=2.0)
    a = ap.parse_args()
    import datetime

    import numpy as np
    import torch.distributed as dist

    from llmctl.serve.control import PeerLostError, ShmChannel

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world,
                            timeout=datetime.timedelta(seconds=60))
    ch = ShmChannel(None, slot_bytes=1 << 16, timeout_s=a.timeout)
    print(f"rank {a.rank} ready pid {os.getpid()}", flush=True)

    def die():
        sys.stdout.flush()
        os.kill(os.getpid(), signal.SIGKILL if a.mode == "kill" else signal.SIGSTOP)
        time.sleep(3600)  # SIGSTOP: frozen here until the test kills it

    n_plans = 40
    try:
        for i in range(n_plans):
            if a.rank == a.victim and i == 3:
                die()
            if a.rank == 0:
                ch.publish({"op": "decode", "ids": [i], "positions": [i], "slots": [i], "ctx": [1],
                            "bt": np.zeros((1, 2), dtype=np.int32)})
            else:
                plan = ch.receive()
                assert int(plan["ids"][0]) == i
    except PeerLostError as e:
        print(f"rank {a.rank}: PeerLostError: {e}", flush=True)
        os._exit(3)  # no teardown through a group that has a dead member
    print(f"rank {a.rank}: finished without noticing", flush=True)
    os._exit(0)


if __name__ == "__main__":
    raise SystemExit(main())

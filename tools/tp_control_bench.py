#!/usr/bin/env python3
"""TP serving control-plane cost per engine step at world N (CPU, gloo): the round-4 path
(``broadcast_object_list`` of the plan dict) vs the packed-record channels of
``llmctl.serve.control`` (gloo tensors; the /dev/shm ring).  Plans have the shape of a real
decode step (16 sequences, 2k context, block tables of a 4k-token max length) and of a 2048-token
prefill chunk.  Reported per channel: rank 0's publish time and the one-way latency to the
other ranks (send timestamp in the plan, CLOCK_MONOTONIC is system-wide), median / p90 in us.

    python tools/tp_control_bench.py [--world 8] [--iters 400]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def plans(kind):
    rng = np.random.default_rng(0)
    if kind == "decode":
        n = 16
        return {"op": "decode", "ids": rng.integers(0, 32000, n).tolist(), "positions": [2047] * n,
                "slots": rng.integers(0, 1 << 20, n).tolist(), "ctx": [2048] * n,
                "bt": rng.integers(0, 1 << 16, (n, 256)).astype(np.int32)}
    T = 2048
    return {"op": "prefill", "ids": rng.integers(0, 32000, T), "pos": np.arange(T, dtype=np.int32),
            "slots": np.arange(T, dtype=np.int64), "cu": [0, T], "ctx": [T],
            "bt": rng.integers(0, 1 << 16, (1, 256)).astype(np.int32), "last": [T - 1],
            "work": list(range(16)), "doc": np.zeros(T, dtype=np.int32)}


def worker(rank, world, port, iters, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llmctl.serve.control import ShmChannel, TensorChannel

    g = dist.new_group(backend="gloo")
    res = {}
    for kind in ("decode", "prefill"):
        base = plans(kind)
        for name in ("object_list", "tensor", "shm"):
            ch = None if name == "object_list" else TensorChannel(g) if name == "tensor" else ShmChannel(g)
            pub, lat = [], []
            dist.barrier(g)
            for it in range(iters):
                if rank == 0:
                    time.sleep(3e-4)  # a GPU decode step's worth of host idle between plans
                    p = dict(base, stamp=time.perf_counter())
                    t = time.perf_counter()
                    if ch is None:
                        dist.broadcast_object_list([p], src=0, group=g)
                    else:
                        ch.publish(p)
                    pub.append((time.perf_counter() - t) * 1e6)
                else:
                    if ch is None:
                        box = [None]
                        dist.broadcast_object_list(box, src=0, group=g)
                        p = box[0]
                    else:
                        p = ch.receive()
                    lat.append((time.perf_counter() - p["stamp"]) * 1e6)
                    assert p["op"] == base["op"]
            dist.barrier(g)
            if ch is not None:
                ch.close()
            skip = iters // 10
            res[f"{kind}/{name}"] = {"pub": pub[skip:], "lat": lat[skip:]}
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--port", type=int, default=29731)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a.world, a.port, a.iters, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    out = dict(q.get() for _ in ps)
    for p in ps:
        p.join()
    pct = lambda xs, f: sorted(xs)[int(f * (len(xs) - 1))]  # noqa: E731
    for key in out[0]:
        pub = out[0][key]["pub"]
        lat = [x for r in range(1, a.world) for x in out[r][key]["lat"]]
        print(json.dumps({"world": a.world, "plan": key.split("/")[0], "channel": key.split("/")[1],
                          "publish_us_p50": round(statistics.median(pub), 1), "publish_us_p90": round(pct(pub, 0.9), 1),
                          "latency_us_p50": round(statistics.median(lat), 1), "latency_us_p90": round(pct(lat, 0.9), 1)}))


if __name__ == "__main__":
    main()

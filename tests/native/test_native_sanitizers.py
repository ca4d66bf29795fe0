"""Host-side sanitizer runs of the native C++ runtime.

The runtime (KV block allocator + sequence tables, prefetching token loader, JSON/text
indexer) is rebuilt with ``-fsanitize=address,undefined`` (resp. ``thread``) into a temp dir
and driven from a child Python process with the sanitizer runtime preloaded; any report
fails the test.  GPU code is not covered (GPU ASan is unavailable on the MI355X pool).
"""

import os
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[2]

DRIVER = textwrap.dedent(r'''
    import importlib.util, sys, json
    import numpy as np
    spec = importlib.util.spec_from_file_location("_llmctl_native", sys.argv[1])
    m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
    tmp = sys.argv[2]
    # block allocator / KV manager: allocate, fork (refcount), append across block edges, free
    kv = m.KVManager(64, 16)
    for s in range(8):
        kv.add_sequence(s, 20 + s)
    kv.fork(0, 100)
    for s in range(8):
        for _ in range(30):
            if kv.can_allocate(1):
                kv.append_token(s)
    tabs = kv.block_tables(list(range(8)), 16)
    for s in list(range(8)) + [100]:
        kv.free_sequence(s)
    assert kv.num_free_blocks == kv.num_blocks
    # token loader: prefetch thread, epoch roll-over, seek
    toks = (np.arange(5000) % 251).astype(np.uint16)
    toks.tofile(tmp + "/t.bin")
    ld = m.TokenLoader(tmp + "/t.bin", 2, 31, 4, 1, 2, 7, 3)
    for _ in range(50):
        ld.next()
    ld.seek(1, 8)
    a = ld.next()
    assert a.shape == (4, 32)
    del ld
    # indexer: jsonl with unicode escapes / surrogate pairs / empty lines
    with open(tmp + "/d.jsonl", "w") as f:
        f.write(json.dumps({"text": "héllo 😀"}) + "\n\n" + json.dumps({"text": "x" * 3000}) + "\n")
    n = m.index_bytes(tmp + "/d.jsonl", tmp + "/d.bin", tmp + "/d.idx", True)
    print("ok", n)
''')


def _runtime(lib: str) -> str:
    r = subprocess.run(["g++", f"-print-file-name={lib}"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else ""


@pytest.mark.parametrize("mode,lib", [("address", "libasan.so"), ("thread", "libtsan.so")])
def test_native_runtime_under_sanitizer(tmp_path, mode, lib):
    rt = _runtime(lib)
    if not rt:
        pytest.skip(f"{lib} not available")
    from llmctl.native.build import build

    so = tmp_path / "_llmctl_native.so"
    build(force=True, verbose=False, sanitize=mode, out=so)
    drv = tmp_path / "drv.py"
    drv.write_text(DRIVER)
    env = dict(os.environ, LD_PRELOAD=rt + (":" + os.environ["LD_PRELOAD"] if os.environ.get("LD_PRELOAD") else ""),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0")
    r = subprocess.run([sys.executable, str(drv), str(so), str(tmp_path)], capture_output=True, text=True,
                       env=env, timeout=600)
    bad = [k for k in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer") if k in r.stderr]
    assert r.returncode == 0 and not bad and "ok" in r.stdout, r.stderr[-4000:]

"""Dataset indexing (``llmctl admin index``): corpus -> uint16 token file + document index.

Uses the native C++ indexer (``llmctl.native.index_bytes``) when built, else numpy.  The
byte-level tokenizer keeps this offline (no tokenizer downloads); the output is what
``MemmapTokens`` / the native ``TokenLoader`` read.
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Any, Dict, Optional


def index_dataset(src: str, out: Optional[str] = None) -> Dict[str, Any]:
    p = Path(src)
    files = sorted([f for f in p.iterdir() if f.suffix in (".txt", ".jsonl")]) if p.is_dir() else [p]
    if not files:
        raise FileNotFoundError(f"no .txt/.jsonl files in {src}")
    results = []
    for f in files:
        bin_path = Path(out) if (out and len(files) == 1) else f.with_suffix(".bin")
        idx_path = bin_path.with_suffix(".idx")
        from llmctl import native

        m = native.load()
        if m is not None:
            ntok, ndocs = m.index_bytes(str(f), str(bin_path), str(idx_path), f.suffix == ".jsonl")
            impl = "native"
        else:
            from llmctl.io.dataset import tokenize_to_bin

            ntok = tokenize_to_bin(str(f), str(bin_path))
            ndocs = None
            impl = "numpy"
        bin_path.with_suffix(".json").write_text(json.dumps({"dtype": "uint16", "tokens": int(ntok),
                                                             "documents": ndocs, "tokenizer": "bytes"}))
        results.append({"source": str(f), "bin": str(bin_path), "idx": str(idx_path), "tokens": int(ntok),
                        "documents": ndocs, "impl": impl})
    return {"files": results}

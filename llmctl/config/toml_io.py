"""TOML read/write without the ``toml`` package (absent from this image).

Reading: ``tomli`` (TOML 1.0) — with a fallback pre-pass that joins the multi-line inline
tables the reference preset uses (``llama-7b-a100x8.toml:69-73`` is TOML-1.1 syntax).
Writing: a small emitter for the value types the llmctl schemas use (str, int, float,
bool, None -> omitted, lists of scalars, lists of tables, nested tables), producing output
that ``tomli`` round-trips.
"""

from __future__ import annotations

import datetime as _dt
import json
import math
import re
from pathlib import Path
from typing import Any, Dict, List

import tomli


def _join_multiline_inline_tables(text: str) -> str:
    out: List[str] = []
    buf = ""
    depth = 0
    for line in text.splitlines():
        stripped = line.split("#", 1)[0] if '"' not in line else line
        if depth > 0:
            buf += " " + line.strip()
        else:
            buf = line
        depth += stripped.count("{") - stripped.count("}")
        if depth <= 0:
            depth = 0
            # drop trailing commas before a closing brace (TOML 1.1 allows them)
            out.append(re.sub(r",\s*}", " }", buf))
            buf = ""
    if buf:
        out.append(buf)
    return "\n".join(out) + "\n"


def loads_toml(text: str) -> Dict[str, Any]:
    try:
        return tomli.loads(text)
    except tomli.TOMLDecodeError:
        return tomli.loads(_join_multiline_inline_tables(text))


def load_toml(path) -> Dict[str, Any]:
    return loads_toml(Path(path).read_text())


def load_any(path) -> Dict[str, Any]:
    p = Path(path)
    if p.suffix == ".json":
        return json.loads(p.read_text())
    if p.suffix in (".yaml", ".yml"):
        import yaml

        return yaml.safe_load(p.read_text()) or {}
    return load_toml(p)


# ----------------------------------------------------------------------------- writer
_BARE = re.compile(r"[A-Za-z0-9_-]+")


_ESC = {'"': '\\"', "\\": "\\\\", "\b": "\\b", "\t": "\\t", "\n": "\\n", "\f": "\\f", "\r": "\\r"}


def _basic_str(s: str) -> str:
    """A TOML basic string: every character literal (UTF-8) except the quote, the backslash and
    the control characters, which are escaped (JSON's encoder would emit surrogate-pair escapes
    for astral characters and leave U+007F raw, both invalid TOML)."""
    out = []
    for ch in s:
        e = _ESC.get(ch)
        if e is not None:
            out.append(e)
        elif ord(ch) < 0x20 or ord(ch) == 0x7F:
            out.append(f"\\u{ord(ch):04x}")
        else:
            out.append(ch)
    return '"' + "".join(out) + '"'


def _key(k: str) -> str:
    return k if _BARE.fullmatch(k) else _basic_str(k)  # fullmatch: "$" would accept a trailing newline


def _scalar(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        if math.isnan(v):
            return "nan"
        if math.isinf(v):
            return "inf" if v > 0 else "-inf"
        r = repr(v)
        if "e" in r or "E" in r:
            m, e = r.lower().split("e")
            if "." not in m:
                m += ".0"
            return f"{m}e{int(e)}"
        return r
    if isinstance(v, str):
        return _basic_str(v)
    if isinstance(v, (_dt.datetime, _dt.date)):
        return v.isoformat()
    if isinstance(v, (list, tuple)):
        return "[" + ", ".join(_scalar(x) for x in v if x is not None) + "]"
    if isinstance(v, dict):
        return "{ " + ", ".join(f"{_key(k)} = {_scalar(x)}" for k, x in v.items() if x is not None) + " }"
    return _basic_str(str(v))


def _is_table_list(v: Any) -> bool:
    return isinstance(v, (list, tuple)) and len(v) > 0 and all(isinstance(x, dict) for x in v)


def _emit(d: Dict[str, Any], prefix: List[str], out: List[str]) -> None:
    scalars = [(k, v) for k, v in d.items() if v is not None and not isinstance(v, dict) and not _is_table_list(v)]
    tables = [(k, v) for k, v in d.items() if isinstance(v, dict)]
    tlists = [(k, v) for k, v in d.items() if _is_table_list(v)]
    for k, v in scalars:
        out.append(f"{_key(k)} = {_scalar(v)}")
    for k, v in tables:
        path = prefix + [_key(k)]
        out.append("")
        out.append(f"[{'.'.join(path)}]")
        _emit(v, path, out)
    for k, v in tlists:
        path = prefix + [_key(k)]
        for item in v:
            out.append("")
            out.append(f"[[{'.'.join(path)}]]")
            _emit(item, path, out)


def dumps_toml(d: Dict[str, Any]) -> str:
    out: List[str] = []
    _emit(d, [], out)
    text = "\n".join(out).lstrip("\n") + "\n"
    return text


def dump_toml(d: Dict[str, Any], path_or_file) -> None:
    text = dumps_toml(d)
    if hasattr(path_or_file, "write"):
        path_or_file.write(text)
    else:
        Path(path_or_file).write_text(text)

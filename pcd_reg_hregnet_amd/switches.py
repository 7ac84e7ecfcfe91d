"""The one debug flag of the package: ``HREG_SWITCHES``.

The engine and trainer keep module-level switches for their alternative kernel paths (the
fp32-MFMA checker kernels, the layer-wise GEMM paths, experimental variants); every default
is the measured product path.  Tests and A/B tools set the attributes directly
(``engine.B6_L1 = False``); a whole process can be started on a variant with
``HREG_SWITCHES="B6_L1=0,SPLIT_L3=1,L1_LDS_MAX_N=0"`` -- the only environment variable the
package reads besides ``HREG_LIB`` (an alternative build of the library, A/B timing only).

Names no module declares raise at package import (``check``, ADVICE r4: a misspelled or
removed switch used to be ignored silently).  ``PROBE_*`` switches are timing probes that
change results (work skipped or run twice); ``bench.py`` refuses to print a measurement while
one is set unless it is told it runs a probe (``--allow-probes``), and every bench line records
``HREG_SWITCHES`` / ``HREG_LIB`` (``provenance``).
"""
from __future__ import annotations

import os


def _parse(text: str) -> dict:
    out = {}
    for item in filter(None, (t.strip() for t in text.split(","))):
        name, sep, value = item.partition("=")
        if not sep:
            raise ValueError(f"HREG_SWITCHES: expected NAME=VALUE, got {item!r}")
        out[name.strip()] = value.strip()
    return out


_SET = _parse(os.environ.get("HREG_SWITCHES", ""))
_USED: set = set()


def flag(name: str, default: bool) -> bool:
    _USED.add(name)
    v = _SET.get(name)
    return default if v is None else v != "0"


def integer(name: str, default: int) -> int:
    _USED.add(name)
    v = _SET.get(name)
    return default if v is None else int(v)


def text(name: str, default: str = "") -> str:
    _USED.add(name)
    return _SET.get(name, default)


def unknown() -> list:
    """names set in HREG_SWITCHES that no module declared (typos)"""
    return sorted(set(_SET) - _USED)


def check() -> None:
    """Raise on names in HREG_SWITCHES that no module declared (called once every module that
    declares switches is imported: the package __init__)."""
    bad = unknown()
    if bad:
        raise ValueError(f"HREG_SWITCHES names unknown switches {bad} (declared: {sorted(_USED)})")


def probes() -> dict:
    """the PROBE_* switches set to a non-default value (timing probes: results change)"""
    return {k: v for k, v in _SET.items() if k.startswith("PROBE_") and v not in ("", "0")}


def provenance() -> dict:
    """what a measurement ran on besides the tree: the switches and the library override"""
    return {"HREG_SWITCHES": os.environ.get("HREG_SWITCHES", ""),
            "HREG_LIB": os.environ.get("HREG_LIB", "")}

"""The one debug flag of the package: ``HREG_SWITCHES``.

The engine and trainer keep module-level switches for their alternative kernel paths (the
fp32-MFMA checker kernels, the layer-wise GEMM paths, experimental variants); every default
is the measured product path.  Tests and A/B tools set the attributes directly
(``engine.B6_L1 = False``); a whole process can be started on a variant with
``HREG_SWITCHES="B6_L1=0,SPLIT_L3=1,L1_LDS_MAX_N=0"`` -- the only environment variable the
package reads besides ``HREG_LIB`` (an alternative build of the library, A/B timing only).
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


def unknown() -> list:
    """names set in HREG_SWITCHES that no module declared (typos)"""
    return sorted(set(_SET) - _USED)

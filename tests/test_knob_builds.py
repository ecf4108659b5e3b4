"""Every build-time knob left in the product sources compiles at a non-default
value (CPU, no device: hipcc -fsyntax-only for gfx950, which instantiates every
kernel template the launchers use and checks their static_asserts).

The knobs are tuning values that tools/variants.sh sets for GPU A/Bs; losing
code paths of earlier A/Bs are deleted from the source, not kept behind a
switch (their records stay in profiles/).  A knob added to the sources without
an entry here fails test_every_knob_is_listed.
"""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dct-carver_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# knob -> (source file, non-default value)
KNOBS = {
    "DCTE_WG8": ("dcte_kernels.hip", "64"),
    "DCTE_TILE_H": ("dcte_kernels.hip", "64"),
    "DCTE_TILE_H16": ("dcte_kernels.hip", "64"),
    "DCTE_G8": ("dcte_kernels.hip", "16"),
    "DCTE_MIN_WAVES": ("dcte_kernels.hip", "3"),
    "DCTE_MIN_WAVES16": ("dcte_kernels.hip", "3"),
    "DCTE_TSTAMP": ("dcte_kernels.hip", "1"),
    "DCTE_PF2_MAXN": ("dcte_kernels.hip", "2"),
    "DCTE_FIX_DIRECT8": ("dcte_kernels.hip", "128u"),
    "DCTE_FIX_DIRECT4": ("dcte_kernels.hip", "64u"),
    "DCTE_FIX_IL": ("dcte_kernels.hip", "2"),
    "DCTE_EPI_MAX_PX": ("dcte_capi.cpp", "0LL"),
    "DCTE_FIX_GPS": ("dcte_kernels.hip", "1"),
    "DCTE_FIX_MINW": ("dcte_kernels.hip", "3"),
    "DCTE_FIX_MINW_LANES": ("dcte_kernels.hip", "3"),
    "DCTE_FIX_MINW_RGB8": ("dcte_kernels.hip", "3"),
    "DCTE_DENSE_CHUNK": ("dcte_kernels.hip", "8"),
    "DCTE_DENSE_OVERSUB": ("dcte_kernels.hip", "1"),
    "DCTE_DENSE_OVERSUB_MEMO": ("dcte_kernels.hip", "16"),
    "DCTE_DENSE_OVERSUB_MEMO8": ("dcte_kernels.hip", "4"),
    "DCTE_MEMO8_BIG_PX": ("dcte_kernels.hip", "0LL"),
    "DCTE_MEMO_SLOTS": ("dcte_kernels.hip", "64"),
    "DCTE_MEMO_WAYS": ("dcte_kernels.hip", "1"),
    "DCTE_EX_TILE_H": ("dcte_exact.hip", "64"),
    "DCTE_EX_MINW": ("dcte_exact.hip", "1"),
    "DCTE_EX16_MINW": ("dcte_exact.hip", "2"),
    "DCTE_SHIFT_VEC": ("dcte_seam.hip", "1"),
    "DCTE_DP_C": ("dcte_dp.hip", "1"),
    "DCTE_DP_R": ("dcte_dp.hip", "16"),
    "DCTE_DP_Q": ("dcte_dp.hip", "2"),
    "DCTE_DP_NB": ("dcte_dp.hip", "2"),
    "DCTE_CHUNK_ROWS": ("dcte_capi.cpp", "2048"),
    "DCTE_MAX_CHUNKS": ("dcte_capi.cpp", "8"),
    "DCTE_CHUNK_SPLIT": ("dcte_capi.cpp", "4"),
    "DCTE_CHUNK_MIN_ROWS": ("dcte_capi.cpp", "64"),
}

_HEADER_GUARDS = {"DCTE_KERNELS_H", "DCTE_LUMA_H", "DCTE_NORM_H", "DCTE_PIXEL_H", "DCTE_MATH_H",
                  "DCTE_PASSES_H", "DCTE_REF64_H", "DCTE_HD", "DCTE_HD_MEMBER"}


def _sources():
    return [f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h"))]


def test_every_knob_is_listed():
    found = set()
    for f in _sources():
        found |= set(re.findall(r"^#ifndef (DCTE_\w+)", open(os.path.join(CSRC, f)).read(), re.M))
    found -= _HEADER_GUARDS
    assert found == set(KNOBS), f"unlisted {sorted(found - set(KNOBS))}, stale {sorted(set(KNOBS) - found)}"


def _syntax(src, defs):
    cmd = [HIPCC, "-std=c++17", "--offload-arch=gfx950", "-fsyntax-only", "-Wno-unused-command-line-argument",
           "-I" + os.path.join(ROOT, "include"), os.path.join(CSRC, src)] + [f"-D{d}" for d in defs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return r.returncode, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_knobs_compile_at_non_default_values():
    jobs = [(name, src, [f"{name}={val}"]) for name, (src, val) in KNOBS.items()]
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(lambda j: (j[0],) + _syntax(j[1], j[2]), jobs))
    bad = [(n, err) for n, rc, err in res if rc != 0]
    assert not bad, bad

"""Loading the committed golden fixtures (tests/golden) -- data only (.npy, json)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Parity bar (BASELINE.json north_star): 1e-5 relative float tolerance.  The
# absolute floor covers windows whose true AC content is 0: the reference's
# double arithmetic can leave ~1e-17 there.
RTOL = 1e-5
ATOL = 1e-9


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_input(name):
    return np.load(os.path.join(GOLDEN, "inputs", name), allow_pickle=False)


def load_map(name):
    return np.load(os.path.join(GOLDEN, "maps", name), allow_pickle=False)


def load_kat(name):
    return np.load(os.path.join(GOLDEN, "kat", name), allow_pickle=False)


def within_tol(got, ref):
    return np.abs(got.astype(np.float64) - ref) <= RTOL * np.abs(ref.astype(np.float64)) + ATOL

"""CPU check of the seam-update rule of dcte_seam.hip.

After removing seam s from a w x h frame, pixel (x, y) of the new frame keeps
the old energy of (x, y) when x + HR < min s over its window rows, takes the
old energy of (x + 1, y) when x - HL >= max s, and is recomputed otherwise.
Checked here bit-exactly on the kernel's own fp32 arithmetic (tests/emu),
with seams that wander, jump, hug the borders, and for both semantics; the
GPU tests (test_seam.py) then only need device == emulation.
"""
import numpy as np
import pytest

import emu_py as EM
from golden_util import load_input
from seam_util import carve, random_seams, seam_span


@pytest.mark.parametrize("n", [2, 4, 8, 16])
@pytest.mark.parametrize("sem", [0, 1])
def test_unaffected_pixels_move_unchanged(n, sem):
    img = np.ascontiguousarray(load_input("natural_rgb_73x59.npy")[:40, :50])
    h, w = img.shape[:2]
    E0, _, _ = EM.energy_map(img, n, 0.15, 0.85, sem=sem)
    for seam in random_seams(h, w, seed=n + 10 * sem, count=6):
        new = carve(img, seam)
        E1, _, _ = EM.energy_map(new, n, 0.15, 0.85, sem=sem)
        lo, hi, HL, HR = seam_span(seam, w, n, sem)
        xs = np.arange(w - 1)[None, :]
        left = xs + HR < lo[:, None]
        right = np.minimum(xs - HL, w - 2) >= hi[:, None]
        assert not (left & right).any()
        assert np.array_equal(E1[left], E0[:, :-1][left])
        assert np.array_equal(E1[right], E0[:, 1:][right])
        # the recomputed band is narrow: N - 1 + (hi - lo) pixels per row at
        # most (one more when a preview N=2 window clamps onto a last-column seam)
        band = (~left & ~right).sum(1)
        assert (band <= n + (hi - lo)).all()

"""The select form of ComputeThreeMaxima that k_match / k_match_kf use (coeb_match.hip
three_maxima) against the reference's if / else-if chain (ORBmatcher.cc:1602-1638), on histograms
built to tie: the rewrite relies on max1 >= max2 >= max3 holding after every bin, so that each
branch of the chain is one combination of the three tests.  Host-side check of the algebra; the
kernels themselves are compared with the oracle by the -m gpu matcher tests."""
import numpy as np

HISTO_LENGTH = 30


def chain(hist):
    """ORBmatcher::ComputeThreeMaxima as the reference writes it."""
    max1 = max2 = max3 = 0
    ind1 = ind2 = ind3 = -1
    for i, s in enumerate(hist):
        if s > max1:
            max3, max2, max1 = max2, max1, s
            ind3, ind2, ind1 = ind2, ind1, i
        elif s > max2:
            max3, max2 = max2, s
            ind3, ind2 = ind2, i
        elif s > max3:
            max3, ind3 = s, i
    if max2 < 0.1 * max1:
        ind2 = ind3 = -1
    elif max3 < 0.1 * max1:
        ind3 = -1
    return ind1, ind2, ind3


def selects(hist):
    """The kernel's form: three tests per bin, every update a select of the old values."""
    max1 = max2 = max3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(hist):
        g1, g2, g3 = s > max1, s > max2, s > max3
        assert max1 >= max2 >= max3 and (not g1 or g2) and (not g2 or g3)
        max3 = max2 if g2 else (s if g3 else max3)
        i3 = i2 if g2 else (i if g3 else i3)
        max2 = max1 if g1 else (s if g2 else max2)
        i2 = i1 if g1 else (i if g2 else i2)
        max1 = s if g1 else max1
        i1 = i if g1 else i1
    if max2 < 0.1 * max1:
        i2 = i3 = -1
    elif max3 < 0.1 * max1:
        i3 = -1
    return i1, i2, i3


def test_select_form_equals_chain_on_tied_histograms():
    rng = np.random.default_rng(7)
    for trial in range(4000):
        hi = int(rng.choice([1, 2, 3, 5, 40, 700]))        # small ranges force ties
        hist = rng.integers(0, hi + 1, HISTO_LENGTH)
        if trial % 5 == 0:                                 # sparse: most bins empty
            hist[rng.random(HISTO_LENGTH) < 0.8] = 0
        h = [int(v) for v in hist]
        assert selects(h) == chain(h), h


def test_select_form_edge_cases():
    for h in ([0] * HISTO_LENGTH, [5] * HISTO_LENGTH, [0] * 29 + [3], [3] + [0] * 29,
              [1, 10, 1, 10, 1, 10] + [0] * 24, list(range(HISTO_LENGTH)), list(range(HISTO_LENGTH, 0, -1))):
        assert selects(h) == chain(h), h

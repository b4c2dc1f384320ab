"""The property the chain's prefix check rests on (csrc/fps.hip fps_prefix_holds), on the C
oracle's restatement of the reference sampler (oracle/pn2_oracle.c, tf_sampling_g.cu:105-170):
sampling a sampler's picks returns their prefix (SA2's 256 of SA1's 1,024 are SA1's first 256,
SA3's 64 of those their first 64, ...), and an exact tie between a pick and a later point is
where it can fail (the reference's tie order, (k mod 512, k div 512), then prefers the later
point). CPU only; the GPU tests check the kernels against the same oracle."""
import importlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from conftest import PKG_NAME  # noqa: E402


def _oracle():
    from oracle import oracle as O
    return O


def test_sampling_a_sampling_is_its_prefix():
    O = _oracle()
    synth = importlib.import_module(PKG_NAME + ".synth")
    for kind in ("scannet", "uniform"):
        x = synth.batch(range(2), 8192, kind)[0]
        cur = O.gather_point(x, O.fps(x, 1024))
        for m in (256, 64, 16):
            idx = O.fps(cur, m)
            assert (idx == np.arange(m)[None]).all(), (kind, m)
            cur = O.gather_point(cur, idx)


def test_a_tie_breaks_the_prefix():
    O = _oracle()
    synth = importlib.import_module(PKG_NAME + ".synth")
    x = synth.batch(range(2), 8192, "scannet")[0]
    p = O.gather_point(x, O.fps(x, 1024))
    p[:, 700] = p[:, 200]  # ties with pick 200 at its step; thread 700 - 512 = 188 < 200 wins
    idx = O.fps(p, 256)
    assert (idx[:, :200] == np.arange(200)[None]).all()
    assert (idx[:, 200] == 700).all()

"""The culled SA1 / MSG samplers' slot -> cell map (csrc/fps_cull.h, `cellof`): the cold waves
on the hot wave's SIMD hold fewer cells. The map is restated here from the kernel's formula and
checked to hold every cell once, with the valid slots on cells [0, NCELL - dropped) and every
cell of a cloud (N <= NPTS) on a valid slot -- the condition under which the picks cannot depend
on the layout (the GPU parity tests check the picks themselves)."""
import pytest

K_WAVE = 64


def layout(NW, PPT, NPTS, PPC, mask=None, D=None):
    NCW, CP = NW - 1, K_WAVE * PPC
    NCELL = NCW * PPT
    if mask is None:  # the kernel's default: cold waves on SIMD 0 (waves 4, 8, 12, ...)
        mask = sum(1 << c for c in range(NCW) if (c + 1) % 4 == 0)
        spare = NCELL - (NPTS + CP - 1) // CP
        nlw = bin(mask).count("1")
        want = 2 if PPC == 1 else 1  # the MSG size (two points per lane per cell) drops one
        D = 0 if nlw == 0 else min(want, spare // nlw)
    nL = bin(mask).count("1") if D > 0 else 0
    cells = {}
    for cw in range(NCW):
        lb = bin(mask & ((1 << cw) - 1)).count("1")
        light = (mask >> cw) & 1
        for s in range(PPT):
            if nL == 0 or s < PPT - D:
                c = s * NCW + cw
            else:
                q = s - (PPT - D)
                c = s * NCW - nL * q + cw - lb if not light else NCELL - nL * D + q * nL + lb
            cells[(s, cw)] = (c, not (light and s >= PPT - D))
    return NCELL, CP, nL * D, cells


@pytest.mark.parametrize("NW,PPT,NPTS,PPC,dropped_want,simd_want",
                         [(16, 9, 8192, 1, 6, [21, 36, 36, 35]),
                          (16, 9, 16384, 2, 3, [24, 35, 35, 34])])
def test_default_layout_is_a_bijection(NW, PPT, NPTS, PPC, dropped_want, simd_want):
    NCELL, CP, dropped, cells = layout(NW, PPT, NPTS, PPC)
    # SA1: waves 4, 8, 12 hold 7 cells each instead of 9; MSG: 8
    assert sorted(c for c, _ in cells.values()) == list(range(NCELL))
    valid = sorted(c for c, v in cells.values() if v)
    assert valid == list(range(NCELL - dropped))
    assert (NCELL - dropped) * CP >= NPTS  # every point of a full cloud sits in a valid slot
    per_simd = [0] * 4
    for (s, cw), (c, v) in cells.items():
        if v and c * CP < NPTS:
            per_simd[(cw + 1) % 4] += 1
    assert dropped == dropped_want
    assert per_simd == simd_want


@pytest.mark.parametrize("mask,D", [(0, 0), (0x088, 3), (0x7000, 2), (0x888, 1)])
def test_ab_layouts_are_bijections(mask, D):
    NCELL, CP, dropped, cells = layout(16, 9, 8192, 1, mask, D)
    assert sorted(c for c, _ in cells.values()) == list(range(NCELL))
    assert sorted(c for c, v in cells.values() if v) == list(range(NCELL - dropped))
    if mask == 0:  # the original layout: slot s of cold wave cw is cell s * NCW + cw
        assert all(c == s * 15 + cw for (s, cw), (c, _) in cells.items())

"""CPU: every form rule of the forward launch (of-spmm_amd/csrc/spmm_launch.h, launch_typed in
spmm_csr_impl.h; DESIGN.md §3 "forms") on both sides of its threshold, through
ofx_spmm_csr_describe (the configuration a launch would take; nothing is launched, so no GPU is
needed).  The GPU tests (test_gpu_forms.py) then run the same launches and compare the bits."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "of-spmm_amd"))

from oneflow_spmm import ops  # noqa: E402

K_SMALL_ROWS = 32768
K_SMALL_NNZ = 1 << 17
K_SMALL_ELEMS = 1 << 23
K_MID_ELEMS = 1 << 28
K_PREFETCH_NNZ = 3 << 20
F32, BF16, F16, F64 = torch.float32, torch.bfloat16, torch.float16, torch.float64


def form(m, nnz, n, dt=F32, idx=torch.int32, **kw):
    return ops.describe(m, kw.pop("k", m), n, nnz, dt, idx, **kw)


def test_small_form_bounds():
    # rows, nonzeros and products (nnz * n) all bound the one-kernel form
    assert form(K_SMALL_ROWS, K_SMALL_NNZ, 16)["form"] == "small"
    assert form(K_SMALL_ROWS + 1, K_SMALL_NNZ, 16)["form"] != "small"
    assert form(K_SMALL_ROWS, K_SMALL_NNZ + 1, 16)["form"] == "mid"
    assert form(20000, K_SMALL_ELEMS // 128, 128)["form"] == "small"
    assert form(20000, K_SMALL_ELEMS // 128 + 1, 128)["form"] == "mid"
    assert form(2708, 10556, 16)["kernel"] == "small"  # Cora-shaped


def test_mid_form_bounds():
    assert form(K_SMALL_ROWS, K_MID_ELEMS // 128, 128)["form"] == "mid"
    above = form(K_SMALL_ROWS, K_MID_ELEMS // 128 + 1, 128)
    assert above["form"] == "narrow" and above["BI"] == 0 and above["PF"] == 1
    assert form(K_SMALL_ROWS + 1, 400_000, 64)["form"] == "narrow"  # rows bound it too (the
    assert form(K_SMALL_ROWS + 1, 400_000, 256)["form"] != "mid"     # prefetching range)


@pytest.mark.parametrize("n", [32, 64, 128])
def test_prefetch_form_bound(n):
    m = 120_000
    below, above = form(m, K_PREFETCH_NNZ, n), form(m, K_PREFETCH_NNZ + 1, n)
    # up to 128 columns: the shifted window with 32-lane wave items ("narrow", round 5)
    assert below["form"] == "narrow" and below["PF"] == 1 and below["WH"] == 1
    assert above["form"] == "bandwidth" and above["PF"] == 0 and above["U"] == 8


def test_narrow_form_n16_fp32():
    m = 169_343
    below, above = form(m, K_PREFETCH_NNZ, 16), form(m, K_PREFETCH_NNZ + 1, 16)
    assert below["form"] == above["form"] == "narrow"
    # below kPrefetchNnz: the mid-width shape with LDS-exchanged wave items (round 5)
    assert (below["VEC"], below["LPR"], below["U"], below["HL"], below["HU"], below["XL"]) == \
        (4, 4, 8, 8, 8, 1)
    assert (above["VEC"], above["LPR"], above["U"], above["HL"], above["HU"]) == (2, 8, 8, 16, 8)
    # above kPrefetchNnz fp32 only (16-bit N = 16 below it: test_narrow_rows_of_mid_size_launches),
    # N = 16 only, 16-B aligned only
    assert form(m, K_PREFETCH_NNZ + 1, 16, BF16)["form"] != "narrow"
    assert form(m, K_PREFETCH_NNZ, 129)["HL"] == 0
    assert form(m, K_PREFETCH_NNZ + 1, 32)["form"] == "bandwidth"
    unaligned = form(m, K_PREFETCH_NNZ, 16, b_addr=260)  # the mid-width shape, shifted windows
    assert (unaligned["VEC"], unaligned["LPR"], unaligned["SH"]) == (4, 4, 1), unaligned


def test_shifted_window_bandwidth_only():
    m, big = 120_000, K_PREFETCH_NNZ + 1
    sh = form(m, big, 99)
    assert sh["SH"] == 1 and sh["VEC"] == 4 and sh["LPR"] == 32
    assert form(m, big, 100)["SH"] == 0
    assert form(m, big, 63)["SH"] == 0  # 17-63 columns: one element per lane
    assert form(m, big, 99, b_addr=260)["SH"] == 1  # 16-B accesses at 4-B alignment
    with pytest.raises(ops._lib.OfxError):  # an fp32 view off 4-B alignment has no lane layout
        form(m, big, 99, b_addr=258)
    # round 5: 16-bit widths above 64 that are not a multiple of 8 (8-element windows, 2-B aligned)
    for dt in (BF16, F16):
        for n, lpr in ((65, 16), (98, 16), (99, 16), (127, 16), (255, 32), (301, 64)):
            d = form(m, big, n, dt)
            assert (d["form"], d["SH"], d["VEC"], d["LPR"]) == ("bandwidth", 1, 8, lpr), (dt, n, d)
            assert form(m, big, n, dt, b_addr=258, c_addr=262)["SH"] == 1
        assert form(m, big, 104, dt)["SH"] == 0 and form(m, big, 104, dt)["VEC"] == 8
        assert form(m, big, 64, dt)["SH"] == 0 and form(m, big, 32, dt)["SH"] == 0


def test_narrow16_lanes():
    m, big = 120_000, K_PREFETCH_NNZ + 1
    for n, vec in ((8, 1), (16, 1), (32, 2), (64, 4), (128, 8)):
        d = form(m, big, n, BF16)
        assert d["form"] == "bandwidth" and d["VEC"] == vec and d["SH"] == 0, (n, d)
    # round 5: the other widths of 17-63 columns in shifted windows (4 elements to 31, 8 above)
    for n, vec, lpr in ((17, 4, 8), (24, 4, 8), (31, 4, 8), (33, 8, 8), (48, 8, 8), (63, 8, 8)):
        d = form(m, big, n, BF16)
        assert (d["form"], d["VEC"], d["LPR"], d["SH"]) == ("bandwidth", vec, lpr, 1), (n, d)


def test_bandwidth_narrow_rows_take_eight_lanes():
    m, big = 120_000, K_PREFETCH_NNZ + 1
    for n in (1, 2, 3, 4, 7):
        d = form(m, big, n)
        assert d["VEC"] == 1 and d["LPR"] == 8, (n, d)
    assert form(m, big, 16, b_addr=260)["LPR"] == 16


def test_cache_hint_and_global_loads():
    # non-temporal col/val/C streams once B exceeds 1 GiB; global B loads from 4 GiB
    assert form(2_449_029, 123_718_280, 128)["NT"] == 1
    assert form(1_000_000, 20_000_000, 64)["NT"] == 0
    papers = form(111_059_956, 1_615_685_872, 128)
    assert papers["BUF"] == 0 and papers["form"] == "bandwidth"


def test_row_range_uses_its_share_of_nonzeros():
    # an 8-way S(0) slice of products is planned as the launch it is (launch_nnz): 1/8 of the
    # nonzeros, still above kPrefetchNnz
    m, nnz = 2_449_029, 123_718_280
    d = form(m, nnz, 128, row_begin=0, row_end=m // 8)
    assert d["form"] == "bandwidth"
    # a small slice of a mid-size graph drops to the prefetching or mid form
    d = form(169_343, 1_166_243, 128, row_begin=0, row_end=40_000)
    assert d["PF"] == 1 and d["form"] == "narrow"  # the prefetching range's mid-width shape


def test_row_range_with_its_known_nonzeros():
    """options.range_nnz: a caller that knows the range's count overrides the
    proportional estimate, e.g. the first eighth of a degree-sorted products graph holding most of
    its nonzeros takes the bandwidth form, a sparse tail slice the prefetching one; the count is
    clamped to the matrix's nnz and 0 keeps the estimate."""
    m, nnz = 2_449_029, 123_718_280
    rng = dict(row_begin=0, row_end=m // 8)
    est = form(m, nnz, 128, **rng)
    assert form(m, nnz, 128, options=ops.make_options(range_nnz=0), **rng) == est
    assert form(m, nnz, 128, options=ops.make_options(range_nnz=2_000_000), **rng)["PF"] == 1
    arxiv = dict(row_begin=0, row_end=30_000)  # estimated 206k nonzeros: the mid form
    assert form(169_343, 1_166_243, 64, **arxiv)["form"] == "mid"
    assert form(169_343, 1_166_243, 64, options=ops.make_options(range_nnz=100_000),
                **arxiv)["form"] == "small"
    assert form(169_343, 1_166_243, 64, options=ops.make_options(range_nnz=10**12),
                **arxiv)["form"] == "mid"  # clamped to the matrix's 1.17M
    # a launch over every row ignores it (nnz is exact there)
    assert form(m, nnz, 128, options=ops.make_options(range_nnz=5))["form"] == "bandwidth"


def test_forced_forms():
    m, nnz = 169_343, 1_166_243
    assert form(m, nnz, 64, options=ops.make_options(variant=30000))["form"] == "small"
    assert form(m, nnz, 64, options=ops.make_options(variant=30001))["form"] == "mid"
    assert form(m, nnz, 64, options=ops.make_options(variant=30003))["form"] == "bandwidth"
    w = form(m, nnz, 64, options=ops.make_options(variant=30004))
    p = form(m, nnz, 64, options=ops.make_options(variant=30005))
    assert w["form"] == p["form"] == "prefetch" and w["WH"] == 1 and p["WH"] == 0
    assert form(m, nnz, 64, options=ops.make_options(variant=416)) == \
        {**form(m, nnz, 64, options=ops.make_options(variant=416)), "VEC": 4, "LPR": 16}


def test_prefetch_form_layouts():
    """The prefetching form's lane layouts (round 4): odd fp32 widths above 16 take 16-B lanes
    with the shifted last window; 16-bit rows of <= 128 B take N / 16 elements per lane."""
    m, nnz = 169_343, 1_166_243
    # above 128 columns: the shifted 16-B window of the prefetching form
    for n, lpr in ((129, 64), (255, 64)):
        d = form(m, nnz, n)
        assert d["SH"] == 1 and d["VEC"] == 4 and d["LPR"] == lpr and d["HL"] == 0, d
        assert d["form"] == ("prefetch" if lpr < 64 else "bandwidth"), d  # 64 lanes: one row a wave
    assert form(m, nnz, 17, b_addr=258 + 2)["SH"] == 1
    for dt in (BF16, F16):
        d = form(m, nnz, 257, dt)  # above 256 columns: 8-element shifted windows
        assert d["SH"] == 1 and d["VEC"] == 8 and d["HL"] == 0, (dt, d)
        assert form(m, nnz, 512, dt)["VEC"] == 8


def test_narrow_rows_of_mid_size_launches():
    """16-bit N = 8 / 16 and fp32 N = 8 in the prefetching form's size range: round 4's narrow
    shape (4 lanes per light row, 16-lane wave items) gave way in round 5 to the mid-width shape
    with LDS-exchanged 8-lane wave items of 2 elements, aligned or not; the sizes either side
    keep their forms."""
    m, nnz = 169_343, 1_166_243
    for dt in (BF16, F16):
        for n in (8, 16):
            d = form(m, nnz, n, dt)
            assert (d["form"], d["VEC"], d["LPR"], d["U"], d["HL"], d["HV"], d["XL"], d["LR"]) == \
                ("narrow", 4, 4, 8, 8, 2, 1, 1), (dt, n, d)
        d = form(m, nnz, 16, dt, b_addr=258)  # 2-B aligned B: the mid-width shape
        assert (d["form"], d["VEC"], d["LPR"], d["SH"]) == ("narrow", 4, 4, 1), d
        # 17-64 columns: launch_mid_width_pf (test_mid_width_rule)
        assert form(m, K_PREFETCH_NNZ + 1, 16, dt)["form"] == "bandwidth"
        assert form(20_000, 400_000, 16, dt)["form"] == "mid"
    d = form(m, nnz, 8)  # round 5: the mid-width shape (LDS-exchanged wave items)
    assert (d["form"], d["VEC"], d["LPR"], d["U"], d["HL"], d["XL"]) == ("narrow", 4, 4, 8, 8, 1), d
    d = form(m, nnz, 8, b_addr=260)  # 4-B aligned B: the mid-width shape
    assert (d["form"], d["VEC"], d["LPR"], d["SH"]) == ("narrow", 4, 4, 1), d
    assert form(m, nnz, 4)["form"] == "narrow"


def test_in_kernel_hub_reduce_only_in_mid_size_forms():
    """Cfg::LR (hub partials added by the last chunk inside spmm_main) in the mid, prefetching and
    narrow-prefetching forms; the bandwidth form keeps the spmm_reduce launch."""
    assert form(20_000, 400_000, 64)["LR"] == 1                 # mid
    assert form(169_343, 1_166_243, 64)["LR"] == 1              # prefetching
    assert form(169_343, 1_166_243, 16)["LR"] == 1              # narrow, <= kPrefetchNnz
    assert form(1_000_000, 20_000_000, 16)["LR"] == 0           # narrow, past it
    assert form(2_449_029, 123_718_280, 128)["LR"] == 0         # bandwidth
    assert form(2708, 10556, 16)["LR"] == 0                     # small form: no plan


def test_mid_width_rule():
    """Round 5 (launch_mid_width_pf): rows of 1-128 columns (fp32) / 1-256 (16-bit) of mid-size
    launches, any width and any element-aligned view (8 / 16 aligned columns too since the
    LDS-exchanged wave items, Cfg::XL, up to 64 columns): shifted windows (one element per lane below 4 columns) with wave items of HL
    lanes x HV elements, one column pass, hubs added in the kernel.  Both sides of every bound:
    3 / 4, 16 / 17, 32 / 33, 64 / 65, 128 / 129, 256 / 257 columns, kPrefetchNnz, the mid / small
    forms below, f64."""
    m, nnz = 169_343, 1_166_243
    for dt in (F32, BF16, F16):
        top = 128 if dt == F32 else 256
        for n in (1, 2, 3, 4, 5, 7, 8, 9, 12, 15, 16, 17, 18, 24, 25, 31, 32, 33, 40, 41, 47, 48, 57, 63,
                  64, 65, 99, 127, 128, 129, 200, 255, 256):
            if n > top:
                continue
            d = form(m, nnz, n, dt)
            if n < 4:
                want = ("narrow", 0, 1, 4, 8, 4, 1, 1)
            elif n <= 16:
                want = ("narrow", 1, 4, 4, 8, 8, 2, 1)
            elif n <= 32:
                want = ("narrow", 1, 4, 8, 8, 8, 4, 1)
            elif n <= 64:
                want = ("narrow", 1, 4, 16, 8, 16, 4, 1) if dt == F32 else ("narrow", 1, 8, 8, 8, 16, 4, 1)
            elif n <= 128:
                want = ("narrow", 1, 8, 16, 8, 32, 4, 1)
            else:
                want = ("narrow", 1, 8, 32, 8, 32, 8, 1)
            got = (d["form"], d["SH"], d["VEC"], d["LPR"], d["U"], d["HL"], d["HV"], d["LR"])
            assert got == want, (dt, n, d)
            assert d["XL"] == (1 if n <= 64 or dt == F32 else 0), (dt, n, d)
            # element-aligned views with odd offsets and strides take the same configuration
            e = 2 if dt != F32 else 4
            v = form(m, nnz, n, dt, b_addr=256 + e, c_addr=256 + 3 * e, ldb=n + 3, ldc=n + 1)
            assert (v["form"], v["VEC"], v["LPR"], v["HL"], v["HV"]) == got[:1] + got[2:4] + got[5:7], v
        assert form(m, nnz, top + 1, dt)["HL"] == 0              # past the rule's widths
        assert form(m, K_PREFETCH_NNZ + 1, 41, dt)["form"] == "bandwidth"
        assert form(20_000, 400_000, 41, dt)["form"] == "mid"
        assert form(19_717, 88_648, 41, dt)["form"] == "small"
    assert form(m, nnz, 41, F64)["HV"] == 1 and form(m, nnz, 41, F64)["form"] != "narrow"



def test_narrow16_lanes_in_small_and_mid_forms():
    """Round 4: 16-bit rows of <= 64 columns take N / 16 elements per lane in the small and mid
    forms too (profiles/r04y_small16.jsonl: PubMed-shaped bf16 N = 8-32 33 -> 23 us)."""
    for dt in (BF16, F16):
        for n, vec in ((8, 1), (16, 1), (32, 2), (64, 4)):
            small = form(19_717, 88_648, n, dt)
            assert small["form"] == "small" and small["VEC"] == vec, (dt, n, small)
            mid = form(20_000, 400_000, n, dt)
            assert mid["form"] == "mid" and mid["VEC"] == vec, (dt, n, mid)
        assert form(19_717, 88_648, 128, dt)["VEC"] == 8  # past 64 columns: the widest vector

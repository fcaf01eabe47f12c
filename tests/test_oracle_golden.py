"""CPU: pin the oracle against the reference's own outputs (golden fixtures).

The fixtures come from running the reference core/corr.py here
(tests/golden/make_golden.py).  These tests establish that the numpy
restatement in oracle/ IS the reference's algorithm, so GPU tests may use it as
the checker at sizes and for inputs the fixtures do not cover.
"""
from __future__ import annotations

import numpy as np
import pytest

import datagen as dg
import oracle
from conftest import load_large, load_tiny, tiny_cases, tolerance_check


def test_generator_is_pinned():
    """Inputs are regenerated from seeds on the GPU box: the stream must not drift."""
    assert dg.splitmix64(0, 3).tolist() == [16294208416658607535, 7960286522194355700,
                                            487617019471545679]
    np.testing.assert_array_equal(dg.uniform(7, 3), [0.3898297483912715, 0.01678829452815611,
                                                      0.9007606806068834])
    np.testing.assert_allclose(dg.normal(0, 4), [2.044272163028782, 1.045091417389922,
                                                 0.34268650712041837, -0.1933658650337396],
                               rtol=1e-15)
    np.testing.assert_array_equal(dg.fmap(1, 1, 2, 2, 2)[0, 0],
                                  np.array([[-1.2145813, 0.13394034], [1.9091979, -1.0727307]],
                                           dtype=np.float32))


@pytest.mark.parametrize("name", tiny_cases())
def test_oracle_pyramid(name):
    d = load_tiny(name)
    rows = d["pyr_rows"]
    p32 = oracle.corr_pyramid(d["fmap1"], d["fmap2"], d["num_levels"], np.float32)
    p64 = oracle.corr_pyramid(d["fmap1"], d["fmap2"], d["num_levels"], np.float64)
    for lvl in range(d["num_levels"]):
        ref = d[f"pyr{lvl}"]
        # float32 mirror: same op sequence; bit-exact on this host's BLAS, so allow
        # only a last-ulp difference for other BLAS kernels.
        tolerance_check(p32[lvl][rows], ref, 1e-6)
        tolerance_check(p64[lvl][rows].astype(np.float32), ref, 1e-5)


@pytest.mark.parametrize("name", [n for n in tiny_cases()
                                  if load_tiny(n)["pyr_rows"].size == load_tiny(n)["B"] *
                                  load_tiny(n)["H"] * load_tiny(n)["W"]])
def test_oracle_lookup_bitexact_on_reference_pyramid(name):
    """corr_lookup on the reference's pyramid reproduces the reference's bits
    (grid_sample coordinate round trip and fused tap sum included)."""
    d = load_tiny(name)
    pyr = [d[f"pyr{lvl}"] for lvl in range(d["num_levels"])]
    for k in range(d["n_coords"]):
        got, ref = oracle.corr_lookup(pyr, d[f"coords{k}"], d["radius"]), d[f"out{k}"]
        assert got.dtype == np.float32 and got.shape == ref.shape
        assert np.array_equal(np.isnan(got), np.isnan(ref))
        fin = ~np.isnan(ref)
        assert np.array_equal(got[fin], ref[fin])


@pytest.mark.parametrize("name", tiny_cases())
def test_oracle_float64_path(name):
    d = load_tiny(name)
    pyr = oracle.corr_pyramid(d["fmap1"], d["fmap2"], d["num_levels"], np.float64)
    for k in range(d["n_coords"]):
        tolerance_check(oracle.corr_lookup(pyr, d[f"coords{k}"], d["radius"]), d[f"out{k}"], 1e-5)


def test_nan_level_is_reference_behaviour():
    """A 1-row/1-column level divides by zero in bilinear_sampler: all NaN."""
    d = load_tiny("nanlevel")
    assert d["pyr3"].shape[-2:] == (1, 2)
    for k in range(d["n_coords"]):
        out = d[f"out{k}"].reshape(1, 4, 81, 12, 16)
        assert np.isnan(out[:, 3]).all() and not np.isnan(out[:, :3]).any()


def _alt_kernel_literal(f1, f2, coords, r):
    """Pure-Python restatement of correlation_kernel.cu:59-114 for ONE query and
    one coordinate set: cell loop iy-major, each dot scattered (+=) to <= 4 taps."""
    rd = 2 * r + 1
    out = np.zeros(rd * rd)
    x, y = np.float32(coords[0]), np.float32(coords[1])
    # scalar_t = float in the kernel (:67-68): x - floor(x) rounds for small negative x
    dx, dy = float(x - np.floor(x)), float(y - np.floor(y))
    H2, W2, _ = f2.shape
    for iy in range(rd + 1):
        for ix in range(rd + 1):
            h2 = int(np.floor(y)) - r + iy
            w2 = int(np.floor(x)) - r + ix
            s = float(f1 @ f2[h2, w2]) if (0 <= h2 < H2 and 0 <= w2 < W2) else 0.0
            if iy > 0 and ix > 0:
                out[(iy - 1) + rd * (ix - 1)] += s * dy * dx
            if iy > 0 and ix < rd:
                out[(iy - 1) + rd * ix] += s * dy * (1 - dx)
            if iy < rd and ix > 0:
                out[iy + rd * (ix - 1)] += s * (1 - dy) * dx
            if iy < rd and ix < rd:
                out[iy + rd * ix] += s * (1 - dy) * (1 - dx)
    return out


def test_alt_forward_matches_literal_kernel_restatement():
    B, H1, W1, H2, W2, C, N, r = 1, 5, 6, 7, 8, 16, 2, 2
    f1 = dg.normal(1, B * H1 * W1 * C).reshape(B, H1, W1, C)
    f2 = dg.normal(2, B * H2 * W2 * C).reshape(B, H2, W2, C)
    c = (dg.uniform(3, B * N * H1 * W1 * 2).reshape(B, N, H1, W1, 2) * 12 - 2).astype(np.float32)
    got = oracle.alt_corr_forward(f1, f2, c, r)
    for n in range(N):
        for h in range(H1):
            for w in range(W1):
                ref = _alt_kernel_literal(f1[0, h, w], f2[0], c[0, n, h, w], r)
                np.testing.assert_allclose(got[0, n, :, h, w], ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("r", [0, 2, 4])
def test_alt_backward_is_the_adjoint_of_the_forward(r):
    """alt_cuda_corr.backward has no runnable reference here (CUDA-only) and no
    golden; it is pinned to the forward restatement above by linearity: for any
    direction d, <corr_grad, forward(d, fmap2)> = <fmap1_grad, d> and
    <corr_grad, forward(fmap1, d)> = <fmap2_grad, d> (windows partly outside)."""
    B, H1, W1, H2, W2, C, N = 2, 5, 7, 6, 9, 12, 2
    rd = 2 * r + 1
    f1 = dg.normal(11, B * H1 * W1 * C).reshape(B, H1, W1, C)
    f2 = dg.normal(12, B * H2 * W2 * C).reshape(B, H2, W2, C)
    c = (dg.uniform(13, B * N * H1 * W1 * 2).reshape(B, N, H1, W1, 2) * 14 - 3).astype(np.float32)
    g = dg.normal(14, B * N * rd * rd * H1 * W1).reshape(B, N, rd * rd, H1, W1)
    g1, g2, gc = oracle.alt_corr_backward(f1, f2, c, g, r)
    assert g1.shape == f1.shape and g2.shape == f2.shape and not gc.any()
    for seed in (15, 16):
        d1 = dg.normal(seed, f1.size).reshape(f1.shape)
        d2 = dg.normal(seed + 10, f2.size).reshape(f2.shape)
        lhs1 = float((g * oracle.alt_corr_forward(d1, f2, c, r)).sum())
        lhs2 = float((g * oracle.alt_corr_forward(f1, d2, c, r)).sum())
        np.testing.assert_allclose(float((g1 * d1).sum()), lhs1, rtol=1e-11, atol=1e-11)
        np.testing.assert_allclose(float((g2 * d2).sum()), lhs2, rtol=1e-11, atol=1e-11)


def test_alt_block_oracle_matches_reference_corrblock():
    """AlternateCorrBlock == CorrBlock by linearity of pooling:
    the only difference is grid_sample's coordinate round trip (a few ulps)."""
    d = load_tiny("batch2_alt")
    for k in range(d["n_coords"]):
        got = oracle.alt_corr_block(d["fmap1"], d["fmap2"], d[f"coords{k}"], 4, d["radius"])
        tolerance_check(got, d[f"out{k}"], 1e-5)


def test_alt_block_oracle_raises_for_small_fmaps():
    f = dg.fmap(5, 1, 8, 12, 20)
    with pytest.raises(RuntimeError):
        oracle.alt_corr_block(f, f, dg.coords(6, 1, 12, 20), 4, 4)


def test_large_chairs_checksums():
    """Benchmark-shape pin (C1 Chairs 46x62): regenerated inputs + float32 oracle
    vs the reference's checksums and sampled entries."""
    d = load_large("chairs")
    B, D, H, W, r = d["B"], d["D"], d["H"], d["W"], d["radius"]
    f1 = dg.fmap(d["fmap_seeds"][0], B, D, H, W, d["dist"])
    f2 = dg.fmap(d["fmap_seeds"][1], B, D, H, W, d["dist"])
    np.testing.assert_allclose([f1.astype(np.float64).sum(), f2.astype(np.float64).sum()],
                               d["fmap_checksum"], rtol=0, atol=1e-6)
    pyr = oracle.corr_pyramid(f1, f2, 4, np.float32)
    for lvl in range(4):
        flat = pyr[lvl].reshape(-1)
        maxabs = float(d[f"pyr{lvl}_maxabs"])
        assert np.abs(flat[d[f"pyr{lvl}_idx"]] - d[f"pyr{lvl}_val"]).max() <= 1e-6 * maxabs
        np.testing.assert_allclose(flat.astype(np.float64).sum(), d[f"pyr{lvl}_sum"][0],
                                   rtol=1e-6, atol=1e-3)
    mode, scale, seed = d["coords"][0]
    out = oracle.corr_lookup(pyr, dg.coords(int(seed), B, H, W, mode, float(scale)), r)
    maxabs = float(d["out0_maxabs"])
    assert np.abs(out.reshape(-1)[d["out0_idx"]] - d["out0_val"]).max() <= 1e-6 * maxabs


def test_large_hd_sampled_rows():
    """C5 1080p (136x240) pin of the sampled-row oracle the GPU tests use at full
    size: corr_rows_pyramid / corr_lookup_rows / alt_corr_block_queries against
    the reference CorrBlock's sampled entries (tests/golden/large_hd.npz)."""
    d = load_large("hd")
    B, D, H, W, r = d["B"], d["D"], d["H"], d["W"], d["radius"]
    n = H * W
    f1 = dg.fmap(d["fmap_seeds"][0], B, D, H, W, d["dist"])[0]
    f2 = dg.fmap(d["fmap_seeds"][1], B, D, H, W, d["dist"])[0]
    np.testing.assert_allclose([f1.astype(np.float64).sum(), f2.astype(np.float64).sum()],
                               d["fmap_checksum"], rtol=0, atol=1e-6)
    sizes = [(H >> lvl, W >> lvl) for lvl in range(4)]
    for lvl, (h, w) in enumerate(sizes):
        idx = d[f"pyr{lvl}_idx"][:512]
        q, cell = np.divmod(idx, h * w)
        uq, inv = np.unique(q, return_inverse=True)
        rows = oracle.corr_rows_pyramid(f1, f2, uq, lvl + 1, np.float64)[lvl].reshape(len(uq), -1)
        got = rows[inv, cell]
        assert np.abs(got - d[f"pyr{lvl}_val"][:512]).max() <= 1e-5 * float(d[f"pyr{lvl}_maxabs"])
    for k, (mode, scale, seed) in enumerate(d["coords"]):
        c = dg.coords(int(seed), B, H, W, mode, float(scale))[0]
        idx = d[f"out{k}_idx"][:256]
        ch, q = np.divmod(idx, n)
        uq, inv = np.unique(q, return_inverse=True)
        cq = c.reshape(2, n)[:, uq].T
        look = oracle.corr_lookup_rows(oracle.corr_rows_pyramid(f1, f2, uq, 4, np.float64), cq, r)
        alt = oracle.alt_corr_block_queries(f1, f2, c, uq, 4, r, np.float64)
        maxabs = float(d[f"out{k}_maxabs"])
        for got in (look[inv, ch], alt[inv, ch]):
            assert np.abs(got - d[f"out{k}_val"][:256]).max() <= 1e-5 * maxabs


# --------------------------------------------------------------------------- backward
@pytest.mark.parametrize("name", ["bw_basic", "bw_batch2_r3", "bw_d256"])
def test_oracle_backward_matches_reference_autograd(name):
    """The float64 backward restatement (grid_sample scatter, avg-pool chain,
    matmul gradients) reproduces the reference autograd's fmap gradients."""
    from conftest import load_backward
    d = load_backward(name)
    L, r = d["num_levels"], d["radius"]
    pyr = oracle.corr_pyramid(d["fmap1"], d["fmap2"], L, np.float64)
    shapes = [p.shape[-2:] for p in pyr]
    dl = [np.zeros(p.shape) for p in pyr]
    for c, w in zip(d["coords"], d["weights"]):
        for acc, g in zip(dl, oracle.corr_lookup_backward(shapes, c, r, w)):
            acc += g
    df1, df2 = oracle.corr_pyramid_backward(d["fmap1"], d["fmap2"], dl)
    for got, ref in ((df1, d["dfmap1"]), (df2, d["dfmap2"])):
        scale = np.abs(ref).max()
        assert np.abs(got - ref).max() <= 1e-5 * scale


@pytest.mark.parametrize("name", ["fnet", "small_r3", "batch2_alt"])
def test_torch_restatement_matches_reference_forward(name):
    """tests/torch_ref.py (the device-side autograd checker of the GPU backward
    tests) reproduces the reference forward on CPU."""
    import torch
    from torch_ref import TorchCorrBlock
    d = load_tiny(name)
    cb = TorchCorrBlock(torch.from_numpy(d["fmap1"]), torch.from_numpy(d["fmap2"]),
                        num_levels=d["num_levels"], radius=d["radius"])
    for k in range(len(d["coords"])):
        out = cb(torch.from_numpy(d[f"coords{k}"])).numpy()
        ref = d[f"out{k}"]
        assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.parametrize("name", ["motion_basic", "motion_small_b2"])
def test_oracle_motion_conv1x1(name):
    """Lookup + ``F.relu(convc1(corr))`` (core/update.py:90 / :71) against the
    reference encoder's output (tests/golden/make_motion_golden.py)."""
    from conftest import load_motion
    d = load_motion(name)
    pyr = oracle.corr_pyramid(d["fmap1"], d["fmap2"], 4, np.float32)
    corr = oracle.corr_lookup(pyr, d["coords"], d["radius"])
    np.testing.assert_allclose(corr.astype(np.float64).sum(), d["corr_checksum"][0],
                               rtol=1e-6, atol=1e-3)
    got = oracle.motion_conv1x1(corr, d["weight"], d["bias"])
    assert got.shape == d["out"].shape == (d["B"], d["cout"], d["H"], d["W"])
    tolerance_check(got.astype(np.float32), d["out"], 1e-5)
    assert (got == 0).any() and (got > 0).any()   # the ReLU clips part of the output

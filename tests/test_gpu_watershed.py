"""GPU: cpx_watershed_cells (k_watershed.hip) bit-identical to the sequential heap flood
(oracle/ws_oracle.py, pinned to skimage 0.18.3 by tests/golden/watershed_cases.npz): the golden
cases themselves, a batch, full-size 2080^2 FOVs with ~300 touching nuclei, and the status word
(rounds used / -1 when the enqueued rounds cannot reach the fixed point)."""
import os

import numpy as np
import pytest
import torch

import cpx_oracle as orc
import ws_oracle as wo
from cpx._lib import check
from cpx.device import _ptr

pytestmark = pytest.mark.gpu


def _ws_gpu(dev, nuc, corr, ch, d, rounds=(16, 16)):
    B, C, H, W = corr.shape
    td = dev.torch_device
    t_n = torch.from_numpy(np.ascontiguousarray(nuc, np.int32)).to(td)
    t_c = torch.from_numpy(np.ascontiguousarray(corr, np.float32)).to(td)
    cells = torch.full_like(t_n, -7)
    cyto = torch.full_like(t_n, -7)
    status = torch.zeros((B, 8), dtype=torch.int32, device=td)
    check(dev.lib.cpx_watershed_cells(dev.h, _ptr(t_n), _ptr(t_c), B, C, ch, H, W, d, rounds[0], rounds[1],
                                      _ptr(cells), _ptr(cyto), _ptr(status), 8), "cpx_watershed_cells")
    dev.sync()
    return cells.cpu().numpy(), cyto.cpu().numpy(), status[:, 0].cpu().numpy()


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "watershed_cases.npz"))


def test_golden_cases(dev, golden):
    d = int(golden["distance"])
    for n in golden["names_cells"]:
        nuc, corr, ref = golden[f"{n}_nuclei"], golden[f"{n}_corr"], golden[f"{n}_cells"]
        cells, cyto, st = _ws_gpu(dev, nuc[None], corr[None, None], 0, d)
        assert st[0] > 0, (n, st)
        np.testing.assert_array_equal(cells[0], ref, err_msg=str(n))
        np.testing.assert_array_equal(cyto[0], np.where(nuc == 0, ref, 0), err_msg=str(n))


def test_batch_and_channel_select(dev, golden):
    d = int(golden["distance"])
    nuc, corr = golden["cells_512_nuclei"], golden["cells_512_corr"]
    nucs = np.stack([nuc, nuc[::-1].copy(), nuc[:, ::-1].T.copy()])
    corrs = np.stack([corr, corr[::-1], corr[:, ::-1].T])
    C = 3  # the elevation channel is plane 2 of 3; the others are noise
    planes = np.random.default_rng(0).uniform(0, 6e4, (3, C, 512, 512)).astype(np.float32)
    planes[:, 2] = corrs
    cells, cyto, st = _ws_gpu(dev, nucs, planes, 2, d)
    for b in range(3):
        ref, _ = wo.cells_watershed(nucs[b], corrs[b], d)
        assert st[b] > 0
        np.testing.assert_array_equal(cells[b], ref, err_msg=f"fov {b}")


def _synth_fov(H, W, n, seed):
    """~n touching elliptical nuclei (labels in random order, with gaps) and a noisy cell channel."""
    rng = np.random.default_rng(seed)
    nuc = np.zeros((H, W), np.int32)
    lam = np.full((H, W), 300.0, np.float32)
    labels = rng.permutation(np.arange(1, 2 * n + 1))[:n]
    for i in range(n):
        cy, cx = rng.uniform(0, H), rng.uniform(0, W)
        ry, rx = rng.uniform(6, 30, 2)
        th = rng.uniform(0, np.pi)
        s = 2.5 * max(ry, rx)
        y0, y1 = int(max(0, cy - 3 * s)), int(min(H, cy + 3 * s + 1))
        x0, x1 = int(max(0, cx - 3 * s)), int(min(W, cx + 3 * s + 1))
        yy, xx = np.mgrid[y0:y1, x0:x1]
        dy, dx = yy - cy, xx - cx
        u = (dy * np.cos(th) + dx * np.sin(th)) / ry
        v = (-dy * np.sin(th) + dx * np.cos(th)) / rx
        sub = nuc[y0:y1, x0:x1]
        sub[(u * u + v * v <= 1.0) & (sub == 0)] = labels[i]
        lam[y0:y1, x0:x1] += np.float32(rng.uniform(500, 4000)) * np.exp(-(dy * dy + dx * dx) / (2 * s * s)).astype(np.float32)
    corr = (rng.poisson(lam) / np.float32(rng.uniform(0.7, 1.3))).astype(np.float32)
    return nuc, corr


@pytest.fixture(scope="module")
def full_size():
    H = W = 2080
    fovs = [_synth_fov(H, W, 320, 11), _synth_fov(H, W, 260, 12)]
    nuc = np.stack([f[0] for f in fovs])
    corr = np.stack([f[1] for f in fovs])[:, None]
    ref = [wo.cells_watershed(nuc[b], corr[b, 0], 15) for b in range(2)]
    return nuc, corr, ref


def test_full_size_2080(dev, full_size):
    nuc, corr, ref = full_size
    cells, cyto, st = _ws_gpu(dev, nuc, corr, 0, 15)
    print("status (100 x relax rounds + jump rounds):", st.tolist())
    for b in range(2):
        assert st[b] > 0, st
        np.testing.assert_array_equal(cells[b], ref[b][0], err_msg=f"fov {b}")
        np.testing.assert_array_equal(cyto[b], ref[b][1], err_msg=f"fov {b}")
        assert (cells[b] != orc.expand_labels(nuc[b], 15)).sum() > 1000


def test_status_reports_unconverged(dev, full_size):
    nuc, corr, _ = full_size
    _, _, st = _ws_gpu(dev, nuc, corr, 0, 15, rounds=(1, 1))
    assert (st == -1).all(), st


def test_status_reports_unresolved_labels(dev, full_size):
    nuc, corr, _ = full_size
    _, _, st = _ws_gpu(dev, nuc, corr, 0, 15, rounds=(24, 1))  # levels converge, chains do not
    assert (st == -1).all(), st


def test_pipeline_unconverged_watershed_is_a_per_site_failure(dev, monkeypatch):
    """ADVICE r2 / VERDICT r3: a FOV whose Cells flood does not converge is re-run on its own with
    twice the rounds, up to cpx.pipeline.WS_RETRIES times (tests/test_gpu_recovery.py); one still
    not converged after the retries is a failed site (no object rows, FovResults.failed), not a
    failed batch — the reference records a site error and carries on
    (Cellpose_GPU_s3fs.py:225-232).  With one round and no retries (WS_RETRIES = 0: a single re-run
    at two rounds) both FOVs here stay unconverged (they need 16 and 8 rounds)."""
    import cpx.pipeline as pl
    from cpx.pipeline import FovPipeline, PipelineConfig
    from cpx.synth import synth_fovs, synth_illum
    monkeypatch.setattr(pl, "WS_RETRIES", 0)
    H = W = 768
    C, B = 5, 2
    w = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "image-processing-suite_amd",
                     "cpx", "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=H, W=W, C=C, batch=B, ws_rounds=(1, 1), weights=w)
    pipe = FovPipeline(dev, cfg, synth_illum(C, H, W, seed=1))
    # 768^2 FOVs with a plausible nucleus count for that area (synth_fovs' default targets 2080^2)
    raw = synth_fovs(B, C, H, W, dev.torch_device, seed=3, nuclei=(30, 45))
    res = pipe.fetch(pipe.run(raw))
    assert res.seg_stats["n_final"].min() >= 10
    assert res.failed is not None and res.failed.all()
    assert (res.recovered & pl.RECOVER_WS).all()  # the re-run was tried
    for s in ("Nuclei", "Cells", "Cytoplasm"):
        for b in range(B):
            assert len(res.objects[s][b]) == 0 and len(res.feats[s][b]) == 0
            assert res.hdr[s][b]["n_objects"] == 0
    ok = FovPipeline(dev, PipelineConfig(H=H, W=W, C=C, batch=B, weights=w), synth_illum(C, H, W, seed=1))
    res2 = ok.fetch(ok.run(raw))
    assert not res2.failed.any() and all(len(res2.objects["Cells"][b]) > 0 for b in range(B))

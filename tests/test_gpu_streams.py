"""Two FovPipelines on two HIP streams of one GPU (two batches in flight, as bench.py runs
them) give bit-identical results to one pipeline running the batches one after the other:
separate libcpx contexts share no scratch, and every reduction is order-independent or
fixed-order."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))


def _same(a, b):
    assert np.array_equal(a.qc.view(np.uint8), b.qc.view(np.uint8))
    for s in ("Nuclei", "Cells", "Cytoplasm"):
        assert np.array_equal(a.hdr[s].view(np.uint8), b.hdr[s].view(np.uint8)), s
        for x, y in zip(a.objects[s], b.objects[s]):
            assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), s
        for x, y in zip(a.feats[s], b.feats[s]):
            assert np.array_equal(x, y, equal_nan=True), s


@pytest.mark.gpu
@pytest.mark.parametrize("split,exclusive", [("none", ("cpnet", "features")), ("halves", ("cpnet", "features")),
                                             ("halves", ())])
def test_two_streams_match_serial(split, exclusive, monkeypatch):
    """split "halves": the product default (cpx.device.pipeline_streams), each stream on its own
    half of the CUs by a CU mask; exclusive: the stages that wait for the other pipeline's same
    stage (the product's pipeline.STAGE_EXCLUSIVE, and none)."""
    import torch
    import cpx.pipeline as pl
    monkeypatch.setattr(pl, "STAGE_EXCLUSIVE", exclusive)
    from cpx.device import Device, pipeline_streams
    from cpx.pipeline import FovPipeline, PipelineConfig
    from cpx.synth import synth_fovs, synth_illum
    H = W = 1040
    C, B = 5, 2
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    illum = synth_illum(C, H, W, seed=1)
    cfg = PipelineConfig(H=H, W=W, C=C, batch=B, weights=w, max_objects=512)
    streams = pipeline_streams(0, 2, split)
    pipes = []
    for st in streams:
        with torch.cuda.stream(st):
            pipes.append(FovPipeline(Device(0), cfg, illum))
    td = pipes[0].dev.torch_device
    batches = [synth_fovs(B, C, H, W, td, seed=s) for s in (5, 6, 7, 8)]
    torch.cuda.synchronize()
    # serial reference on pipeline 0 / stream 0
    ref = []
    with torch.cuda.stream(streams[0]):
        for x in batches:
            pipes[0].run(x)
            ref.append(pipes[0].fetch())
    torch.cuda.synchronize()
    # interleaved: batch i on pipeline i % 2, both streams busy
    slots = []
    for i, x in enumerate(batches):   # each pipeline holds two steps in its two result slots
        with torch.cuda.stream(streams[i % 2]):
            slots.append(pipes[i % 2].run(x))
    got = [pipes[i % 2].fetch(sl) for i, sl in enumerate(slots)]
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        _same(a, b)

"""BASELINE configs[3]'s job shape at one-box scale: several (plate, time) jobs drained by
several ranks from one work queue.  2 plates x 2 timepoints x 4 wells x 2 sites of 2080 x 2080 x
5-channel synthetic FOVs as uncompressed TIFFs, one LoadData file per (plate, time) job (as
Feature_extraction_opt.py:63-76 fans the plates x times out), through `cpx.launch --gpus 3` with
all three ranks on the test GPU claiming batches from the per-job WorkQueue counters (the
reference's GPU consumers pulling sites from one queue, Cellpose_GPU_s3fs.py:269-300):

  * every <plate>/<time>/ table is byte-identical to a one-process run;
  * two FOVs (of different jobs) equal the CPU path (oracle/cpu_pipeline.run_fov) row for row
    under the rules of tests/test_gpu_config2_full.py (same objects and ObjectNumbers; features
    within rtol 1e-5 except the few objects carrying fp32 rounding-noise boundary pixels);
  * the per-time profiles (cpx.profiles, Pycyto_pertime.py) run over every job.
"""
import filecmp
import os

import numpy as np
import pandas as pd
import pytest
import torch

import cpu_pipeline
from csv_tables import CHANNELS, cpu_tables

pytestmark = pytest.mark.gpu

PLATES = ["P01", "P02"]
TIMES = [6, 24]
WELLS = ["C01", "C02", "C03", "C04"]
SITES = 2


@pytest.mark.timeout(1200)
def test_config3_jobs_three_ranks_work_queue(tmp_path, dev):
    from cpx import launch, plate, profiles, shard, tiffio
    from cpx.cpnet import build_cpnet
    from cpx.csvout import OBJECT_TABLES
    from cpx.synth import synth_fovs, synth_illum
    C, H, W = len(CHANNELS), 2080, 2080
    imgdir, illdir = tmp_path / "images", tmp_path / "illum"
    imgdir.mkdir()
    illdir.mkdir()
    illum = synth_illum(C, H, W, seed=1)
    for c, ch in enumerate(CHANNELS):
        np.save(illdir / f"{ch}_illum.npy", illum[c])
    n = len(WELLS) * SITES
    lds, raws = [], {}
    for plate_id in PLATES:
        for t in TIMES:
            raw = synth_fovs(n, C, H, W, dev.torch_device,
                             seed=shard.fov_seed(shard.Fov(plate_id, "C01", 1, t))).cpu().numpy().view(np.uint16)
            raws[plate_id, t] = raw.reshape(n, C, H, W)
            rows = []
            for wi, well in enumerate(WELLS):
                for s in range(SITES):
                    f = wi * SITES + s
                    row = {"Metadata_Plate": plate_id, "Metadata_Well": well, "Metadata_Site": s + 1,
                           "Metadata_Timepoint": t, "Metadata_Compound": ["DMSO", "CmpA", "DMSO", "CmpB"][wi],
                           "Metadata_ConcLevel": 0 if wi % 2 == 0 else 1}
                    for c, ch in enumerate(CHANNELS):
                        name = f"{plate_id}_t{t}_f{f}_c{c}.tiff"
                        tiffio.imwrite(str(imgdir / name), raws[plate_id, t][f, c])
                        row[f"FileName_{ch}"] = name
                    rows.append(row)
            ld = tmp_path / f"load_data_{plate_id}_{t}.csv"
            pd.DataFrame(rows).to_csv(ld, index=False)
            lds.append(str(ld))
    # batches of 2 FOVs: 4 per job, 16 claims over the 3 ranks
    common = ["--load-data", *lds, "--data-path", str(imgdir), "--illum-path", str(illdir),
              "--channels", *CHANNELS, "--batch", "2", "--threads", "4", "--pipes", "1"]
    three = launch.main(["--gpus", "3", "--devices", "0,0,0", "--", *common, "--out", str(tmp_path / "three")])
    one = plate.run(common + ["--out", str(tmp_path / "one"), "--world", "1", "--rank", "0"])
    jobs = [f"{p}/{t}" for p in PLATES for t in TIMES]
    assert [os.path.relpath(d, tmp_path / "three") for d in three] == jobs
    assert [os.path.relpath(d, tmp_path / "one") for d in one] == jobs
    for d1, d3 in zip(one, three):
        for name in ("Image", *OBJECT_TABLES, "site_status"):
            assert filecmp.cmp(os.path.join(d1, f"{name}.csv"), os.path.join(d3, f"{name}.csv"),
                               shallow=False), (d3, name)
        st = pd.read_csv(os.path.join(d3, "site_status.csv"))
        assert (st.status == "success").all() and len(st) == n
    # the CPU path on two FOVs of two different jobs, every table row
    torch.set_num_threads(16)
    net = build_cpnet(state_dict_path=os.path.join(os.path.dirname(plate.__file__), "weights",
                                                   "cpnet_nuclei_synth.pt"))
    for (plate_id, t), f in ((("P01", 6), 0), (("P02", 24), 5)):
        d = os.path.join(tmp_path / "three", plate_id, str(t))
        gpu = {name: pd.read_csv(os.path.join(d, f"{name}.csv")) for name in ("Image", *OBJECT_TABLES)}
        img_no = f + 1  # LoadData row + 1
        ref = cpu_pipeline.run_fov(raws[plate_id, t][f], illum, net, cell_channel=CHANNELS.index("AGP"))
        cdir = cpu_tables(ref, image_number=img_no).write(str(tmp_path / f"cpu_{plate_id}_{t}"), plate_id, t)
        for name in OBJECT_TABLES:
            c = pd.read_csv(os.path.join(cdir, f"{name}.csv"))
            g = gpu[name][gpu[name].ImageNumber == img_no].reset_index(drop=True)
            assert len(c) == len(g) and len(c) > 100, (name, len(c), len(g))
            np.testing.assert_array_equal(c.ObjectNumber.to_numpy(), g.ObjectNumber.to_numpy())
            feat = [k for k in c.columns if k not in ("ImageNumber", "ObjectNumber")]
            gv, cv = g[feat].to_numpy(np.float64), c[feat].to_numpy(np.float64)
            ok = np.isclose(gv, cv, rtol=1e-5, atol=1e-9) | (np.isnan(gv) & np.isnan(cv))
            off = np.nonzero(~ok.all(axis=1))[0]
            area = feat.index("AreaShape_Area")
            print(plate_id, t, name, "objects beyond rtol 1e-5:", off.tolist(),
                  "area diffs:", (gv[off, area] - cv[off, area]).tolist())
            assert len(off) <= 4, (name, off.tolist())
            assert np.all(np.abs(gv[off, area] - cv[off, area]) <= 8), (name, off.tolist())
        ci = pd.read_csv(os.path.join(cdir, "Image.csv"))
        gi = gpu["Image"][gpu["Image"].ImageNumber == img_no]
        for k in ci.columns:
            if k.startswith("ImageQuality_PercentMaximal") or k.startswith("Count_"):
                assert ci[k].iloc[0] == gi[k].iloc[0], k
            elif k.startswith("ImageQuality_PowerLogLogSlope"):
                assert abs(ci[k].iloc[0] - gi[k].iloc[0]) <= 1e-9 * abs(ci[k].iloc[0]), k
    # per-time profiles (Pycyto_pertime.py) over every job of the queue-drained output
    for plate_id in PLATES:
        written = profiles.concatenate_csv(str(tmp_path / "three"), [str(t) for t in TIMES], plate_id,
                                           str(tmp_path / "prof"), f"{plate_id}_profiles",
                                           local_dir=str(tmp_path / "tmp"))
        assert len(written) == 3 * len(TIMES)

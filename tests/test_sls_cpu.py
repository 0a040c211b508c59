"""SLS data pipeline host logic vs oracle/sls_ref.py: the reference's
valid-piece / label / process-parameter logic (models/CvT(Par).py:363-412), StandardScaler
(pinned against scikit-learn), the train/val split (:437-453), the cv2 INTER_LINEAR axis
tables (host half of the GPU resize), and the workbook reader on the reference's own
workbooks when /root/reference is present (read in place, never copied; skipped elsewhere)."""
import math
import os

import numpy as np
import pytest

from oracle import sls_ref
from vitmi import sls
from vitmi.xlsx import read_xlsx

REF_EXCEL = "/root/reference/Excel"
have_ref = pytest.mark.skipif(not os.path.isdir(REF_EXCEL), reason="reference workbooks absent")


def random_tables(seed, groups=12, per=5, nan_frac=0.15):
    rng = np.random.default_rng(seed)
    lab = rng.normal(1000, 50, groups * per)
    lab[rng.random(groups * per) < nan_frac] = np.nan
    proc = np.stack([rng.choice([1000.0, 500.0], groups), rng.choice([800.0, 1000.0, 1200.0], groups),
                     rng.choice([150.0, 200.0, 250.0], groups), np.full(groups, 0.1),
                     rng.uniform(40, 120, groups)], 1)
    return list(lab), proc.tolist()


@pytest.mark.parametrize("seed,gs,ge,layers", [(0, 1, 12, 3), (1, 3, 10, 4), (2, 1, 12, 1)])
def test_index_and_split_match_oracle(seed, gs, ge, layers):
    lab, proc = random_tables(seed)
    spec = sls.SLSSpec(group_start=gs, group_end=ge, image_layers=layers)
    labels, ps, valid, count = sls.build_index(spec, lab, proc)
    rl, rp, rv, rc = sls_ref.preprocess_index(lab, proc, gs, ge, 1, 5, layers)
    assert count == rc and np.array_equal(valid, rv)
    assert np.array_equal(labels, rl)
    assert np.allclose(ps, rp, rtol=0, atol=1e-12)
    tr, va = sls.split_rows(valid, count, layers)
    rtr, rva = sls_ref.split_train_val(rv, rc, layers)
    assert tr.tolist() == rtr and va.tolist() == rva
    assert len(set(tr.tolist()) | set(va.tolist())) == len(labels)


def test_standard_scaler_matches_sklearn():
    from sklearn.preprocessing import StandardScaler
    _, proc = random_tables(3)
    x = np.repeat(np.asarray(proc), 7, axis=0)
    ref = StandardScaler().fit_transform(x)
    assert np.allclose(sls.standard_scaler(x), ref, rtol=0, atol=1e-12)
    assert np.allclose(sls_ref.standard_scaler(x), ref, rtol=0, atol=1e-12)
    assert np.all(np.abs(ref[:, 3]) < 1e-12)          # the constant hatch-spacing column


@pytest.mark.parametrize("ssize,dsize", [(340, 128), (345, 128), (128, 128), (5, 17), (64, 7), (1, 4)])
def test_resize_tables_match_oracle(ssize, dsize):
    ofs, w = sls.resize_table(ssize, dsize)
    rofs, rw = sls_ref.resize_coeffs(ssize, dsize)
    assert np.array_equal(ofs, rofs) and np.array_equal(w.reshape(-1, 2), rw)


def test_layer_paths_follow_reference_layout():
    spec = sls.SLSSpec(data_root="/d", image_layers=2)
    p = sls.layer_paths(spec, [0, 7, 199])
    assert p[0] == "/d/circle(340x345)/trail1_01/layer_01.jpg"
    assert p[3] == "/d/circle(340x345)/trail2_03/layer_02.jpg"
    assert p[5] == "/d/circle(340x345)/trail40_05/layer_02.jpg"


@have_ref
def test_reference_workbooks():
    s = read_xlsx(os.path.join(REF_EXCEL, "Processed_Circle_test.xlsx"))
    assert s.nrows == 200 and s.header[0] == "Unnamed: 0"
    assert set(sls.FREQUENCIES) <= set(s.header)
    p = read_xlsx(os.path.join(REF_EXCEL, "Process_parameters.xlsx"))
    assert p.header[1:6] == sls.PROCESS_PARAMETERS and p.nrows >= 40
    spec = sls.SLSSpec(labels_xlsx=os.path.join(REF_EXCEL, "Processed_Circle_test.xlsx"),
                       process_xlsx=os.path.join(REF_EXCEL, "Process_parameters.xlsx"))
    for freq in ("50HZ_Bm", "800HZ_Pcv"):
        spec.freq = freq
        labels, proc, valid, count = sls.build_index(spec)
        col = [s.cell(i, freq) for i in range(200)]
        rows = [[p.cell(g, n) for n in sls.PROCESS_PARAMETERS] for g in range(40)]
        rl, rp, rv, rc = sls_ref.preprocess_index(col, rows, 1, 40, 1, 5, 200)
        assert count == 200 == rc and np.array_equal(valid, rv) and np.array_equal(labels, rl)
        assert np.allclose(proc, rp, atol=1e-12)
        assert len(valid) == sum(1 for v in col if not math.isnan(v))
        tr, va = sls.split_rows(valid, count, 200)
        assert len(va) == 200 * len(set(int(v) // 5 for v in valid))   # one validation piece per 5-block
        assert len(tr) + len(va) == len(labels)

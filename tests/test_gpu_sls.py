"""GPU side of SURVEY §8f rows 2-4 against the oracles: the SLS image preprocessing kernel
(cv2 INTER_LINEAR + BGR2GRAY + /255 in OpenCV's 8-bit fixed point, oracle/sls_ref.py) --
bit-exact; the chunked decode->pinned->H2D->kernel loader; device batch gathers; the Keras-style
training loop (Adam, LR schedule, MSE/MAE history, inference-mode validation); weight
save/load; Grad-CAM heatmaps vs the CPU oracle's autograd (fp32, 1e-3)."""
import os

import numpy as np
import pytest
import torch

from oracle import cvt_ref, sls_ref
from vitmi import checkpoint, cvt, gradcam, optim, sls, train

pytestmark = pytest.mark.gpu
DEV = "cuda"


def frames(n, H, W, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:H, 0:W]
    f[0] = np.stack([(xx * 255 // max(W - 1, 1)), (yy * 255 // max(H - 1, 1)), ((xx + yy) % 256)], -1)
    f[-1] = 255 - f[0]
    return f


@pytest.mark.parametrize("n,H,W,Ho,Wo,bgr", [(5, 345, 340, 128, 128, False), (3, 345, 340, 128, 128, True),
                                             (4, 13, 7, 40, 23, False), (2, 64, 64, 64, 64, False),
                                             (3, 100, 90, 33, 47, True)])
def test_sls_preprocess_bit_exact(n, H, W, Ho, Wo, bgr):
    f = frames(n, H, W, n + H)
    out = sls.preprocess_frames(torch.from_numpy(f).to(DEV), Ho, Wo, bgr=bgr).cpu().numpy()
    for i in range(n):
        ref = sls_ref.sls_image(f[i] if bgr else f[i][..., ::-1], Wo, Ho)
        assert np.array_equal(out[i, 0], ref), i


def test_load_images_chunked_pipeline(tmp_path):
    from PIL import Image
    f = frames(7, 345, 340, 3)
    paths = []
    for i in range(7):
        p = str(tmp_path / f"layer_{i + 1:02d}.jpg")
        Image.fromarray(f[i]).save(p, quality=90)
        paths.append(p)
    out = sls.load_images(paths, 128, 128, DEV, chunk=3, workers=4).cpu().numpy()
    for i, p in enumerate(paths):
        rgb = sls.decode_jpeg_rgb(p)
        assert np.array_equal(out[i, 0], sls_ref.sls_image(rgb[..., ::-1]))


def test_gather_rows():
    src = torch.randn(50, 3, 8, 8, device=DEV)
    idx = torch.tensor([3, 0, 49, 7, 7], device=DEV)
    assert torch.equal(sls.gather_rows(src, idx), src[idx])
    s2 = torch.arange(50 * 5, dtype=torch.float32, device=DEV).view(50, 5)      # 20-byte rows: byte path
    assert torch.equal(sls.gather_rows(s2, idx), s2[idx])
    bad = torch.tensor([1, -1, 50], device=DEV)
    g = sls.gather_rows(s2, bad)
    assert torch.equal(g[0], s2[1]) and torch.count_nonzero(g[1:]).item() == 0


def tiny_cfg(method="dw_bn", cls_last=True, proc_dim=5, img=64):
    return cvt.CvTConfig(img_size=img, num_classes=1, proc_dim=proc_dim, dtype="fp32",
                         stages=[cvt.CvTStage(64, 7, 4, 1, qkv_method=method),
                                 cvt.CvTStage(128, 3, 2, 2, qkv_method=method, with_cls_token=cls_last)])


def test_dataset_from_layout_and_batches(tmp_path):
    from PIL import Image
    spec = sls.SLSSpec(data_root=str(tmp_path), group_end=2, image_layers=2, height=64, width=64)
    lab = [1.0, np.nan, 3.0, 4.0, 5.0, 6.0, np.nan, 8.0, 9.0, 10.0]
    proc = [[1000, 1000, 150, 0.1, 60], [500, 800, 200, 0.1, 80]]
    f = frames(20, 69, 68, 9)
    k = 0
    for g in (1, 2):
        for pc in range(1, 6):
            d = tmp_path / f"circle(340x345)/trail{g}_{pc:02d}"
            d.mkdir(parents=True)
            for layer in (1, 2):
                Image.fromarray(f[k]).save(str(d / f"layer_{layer:02d}.jpg"))
                k += 1
    ds = sls.SLSDataset.from_reference_layout(spec, DEV, label_col=lab, process_rows=proc, workers=2)
    assert len(ds) == 16 and ds.images.shape == (16, 1, 64, 64)
    rl, rp, rv, rc = sls_ref.preprocess_index(lab, proc, 1, 2, 1, 5, 2)
    assert np.array_equal(ds.labels.cpu().numpy(), rl.astype(np.float32))
    assert np.allclose(ds.proc.cpu().numpy(), rp.astype(np.float32))
    tr, va = sls_ref.split_train_val(rv, rc, 2)
    assert sorted(ds.val_rows.tolist()) == va and sorted(ds.train_rows.tolist()) == tr
    seen = []
    for img, pr, y in ds.batches(ds.train_rows, 5, shuffle=True, generator=torch.Generator(device=DEV).manual_seed(0)):
        assert img.shape[0] == pr.shape[0] == y.shape[0] <= 5
        for j in range(y.numel()):
            r = int((ds.labels == y[j]).nonzero()[0])
            seen.append(r // 2)
    assert len(seen) == len(tr)


def test_fit_history_schedule_and_checkpoint(tmp_path):
    ds = sls.SLSDataset.synthetic(n_pieces=10, image_layers=6, height=64, width=64, device=DEV)
    torch.manual_seed(0)
    model = cvt.CvT(tiny_cfg()).to(DEV)
    model.reset_parameters(1)
    opt = optim.Adam(list(model.parameters()), learning_rate=1e-3)
    hist = train.fit(model, ds, epochs=3, batch_size=16, optimizer=opt,
                     lr_schedule=lambda e, lr: optim.keras_step_decay(e, lr, every=2), seed=1)
    assert hist["epoch"] == [1, 2, 3] and len(hist["val_loss"]) == 3
    assert hist["lr"] == [1e-3, 1e-3, 1e-3 * 0.8]
    assert hist["loss"][-1] < hist["loss"][0]
    assert opt.iterations == 3 * ((len(ds.train_rows) + 15) // 16)
    train.write_history(hist, str(tmp_path / "h.csv"))
    # save / load (params + BN moving stats + optimizer moments) -> identical inference
    ck = str(tmp_path / "w.safetensors")
    checkpoint.save_weights(model, ck, optimizer=opt)
    m2 = cvt.CvT(tiny_cfg()).to(DEV)
    o2 = optim.Adam(list(m2.parameters()))
    checkpoint.load_weights(m2, ck, optimizer=o2)
    assert o2.iterations == opt.iterations and all(torch.equal(a, b) for a, b in zip(o2._m, opt._m))
    ev1 = train.evaluate(model, ds, ds.val_rows, 16)
    ev2 = train.evaluate(m2, ds, ds.val_rows, 16)
    assert ev1 == ev2 and abs(ev1["loss"] - hist["val_loss"][-1]) < 1e-9
    with pytest.raises(KeyError):
        checkpoint.load_weights(cvt.CvT(tiny_cfg(proc_dim=0)).to(DEV), ck)


@pytest.mark.parametrize("batch_size,cls_last,stage", [(1, False, -1), (2, False, -1), (1, True, 0)])
def test_gradcam_matches_oracle(batch_size, cls_last, stage):
    ocfg = cvt_ref.CvTConfig(img_size=64, num_classes=1, proc_dim=5, dtype="fp32",
                             stages=[cvt_ref.CvTStage(64, 7, 4, 1, qkv_method="avg"),
                                     cvt_ref.CvTStage(128, 3, 2, 2, qkv_method="avg", with_cls_token=cls_last)])
    params = cvt_ref.init_params(ocfg, 4)
    img, _ = cvt_ref.synthetic_batch(ocfg, 4, seed=2)
    proc = cvt_ref.synthetic_proc(ocfg, 4)
    ref = cvt_ref.gradcam(img, params, ocfg, proc, stage=stage, batch_size=batch_size)
    model = cvt.CvT(tiny_cfg("avg", cls_last)).to(DEV)
    model.load_param_dict(params)
    hm = gradcam.gradcam_heatmaps(model, img.to(DEV), proc.to(DEV), stage=stage, batch_size=batch_size, chunk=4)
    assert hm.shape == ref.shape
    assert ((hm.cpu() - ref).norm() / ref.norm()).item() < 1e-3
    assert all(p.grad is None for p in model.parameters())

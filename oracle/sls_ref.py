"""ORACLE — CPU restatement of the reference's SLS data pipeline (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` use this module; the product package never imports it.

SURVEY §8f row 3, ``preprocess_data`` / ``train_and_save_model`` (``models/CvT(Par).py:363-453``):

* labels: column ``freq`` of ``Processed_Circle_test.xlsx``; piece ``count`` (0-based over
  groups 1..group_end x pieces piece_start..piece_end) is valid when its label is not NaN; a
  valid piece inside [start_index, end_index) contributes its label ``image_layers`` times
  (``:375-388``);
* process parameters: the five columns of ``Process_parameters.xlsx`` row ``index // pieces``,
  repeated ``image_layers`` times, then ``StandardScaler().fit_transform`` (``:391-412``);
* images: ``cv2.imread`` (BGR) -> ``cv2.resize(img, (W, H))`` (INTER_LINEAR) ->
  ``cv2.cvtColor(BGR2GRAY)`` -> ``/ 255.0`` (``:414-428``);
* split: the first valid piece of every block of 5 consecutive pieces goes to validation
  (``:437-453``).

The OpenCV functions are a third-party dependency absent here (no cv2 in this image, version
unpinned by the reference).  Restated from OpenCV 4.x's published 8-bit algorithms:

* ``resize`` INTER_LINEAR, 8U (``imgproc/src/resize.cpp``: ``resizeGeneric_`` with
  ``HResizeLinear<uchar,int,short,2048>`` and ``VResizeLinear`` + ``VResizeLinearVec_32s8u``):
  source coordinate ``f = (float)((d + 0.5) * scale - 0.5)``, ``s = floor(f)``, ``f -= s``,
  clamped at the borders; weights ``saturate_cast<short>((1 - f) * 2048)`` and
  ``saturate_cast<short>(f * 2048)``; horizontal pass exact in int32; vertical pass as the SIMD
  kernel computes it: ``((((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16) + 2) >> 2``,
  saturated to uint8 (the scalar tail ``(S0 b0 + S1 b1 + 2^21) >> 22`` can differ by 1 LSB, and
  IPP-accelerated builds may differ too: parity vs cv2 itself is UNPINNED);
* ``cvtColor`` BGR2GRAY, 8U: ``(B*1868 + G*9617 + R*4899 + 2^13) >> 14``.

StandardScaler (scikit-learn, importable here) pins ``standard_scaler``.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np

PROCESS_PARAMETERS = ["氧濃度", "雷射掃描速度", "雷射功率", "線間距", "能量密度"]   # :392


# ---------------------------------------------------------------- labels / process parameters
def preprocess_index(label_col: Sequence[float], process_rows: Sequence[Sequence[float]], group_start: int,
                     group_end: int, piece_start: int, piece_end: int, image_layers: int):
    """models/CvT(Par).py:363-412 as loops.  label_col[count] = label of piece ``count``;
    process_rows[g] = the 5 process parameters of group g (0-based).  Returns (labels
    [n_valid*layers] float64, proc_scaled [n_valid*layers, 5] float64, valid indices, count)."""
    per = piece_end - piece_start + 1
    start_index = (group_start - 1) * per
    end_index = group_end * per
    valid_indices, label_groups = [], []
    count = 0
    for _ in range(1, group_end + 1):
        for _ in range(piece_start, piece_end + 1):
            lab = label_col[count]
            if not (lab is None or (isinstance(lab, float) and math.isnan(lab))):
                if start_index <= count < end_index:
                    label_groups.extend([lab] * image_layers)
                valid_indices.append(count)
            count += 1
    valid = [i for i in valid_indices if start_index <= i < end_index]
    proc = []
    for index in valid:
        proc.extend([list(process_rows[index // per])] * image_layers)
    proc = np.array(proc, dtype=np.float64)
    return np.array(label_groups, dtype=np.float64), standard_scaler(proc), np.array(valid), count


def standard_scaler(x: np.ndarray) -> np.ndarray:
    """StandardScaler().fit_transform: (x - mean) / std (population std; a zero std -> 1)."""
    mean = x.mean(axis=0)
    std = x.std(axis=0)
    std = np.where(std < 10 * np.finfo(np.float64).eps * np.maximum(1.0, np.abs(mean)), 1.0, std)
    return (x - mean) / std


def split_train_val(valid: Sequence[int], count: int, image_layers: int) -> Tuple[List[int], List[int]]:
    """models/CvT(Par).py:437-453: layer-row indices of the training and validation sets."""
    first = []
    valid_set = set(int(v) for v in valid)
    for d in range(0, count, 5):
        for j in range(d, d + 5):
            if j in valid_set:
                first.append(j)
                break
    train, val = [], []
    for i, v in enumerate(valid):
        rows = list(range(i * image_layers, (i + 1) * image_layers))
        (val if int(v) in first else train).extend(rows)
    return train, val


# ---------------------------------------------------------------- images
def resize_coeffs(ssize: int, dsize: int):
    """cv2 INTER_LINEAR source offsets and Q11 weights along one axis."""
    inv_scale = dsize / ssize
    scale = 1.0 / inv_scale
    ofs = np.zeros(dsize, np.int64)
    w = np.zeros((dsize, 2), np.int64)
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0), 0
        if s >= ssize - 1:
            f, s = np.float32(0), ssize - 1
        c0, c1 = np.float32(np.float32(1) - f), f
        w[d, 0] = int(np.rint(np.float32(c0 * np.float32(2048))))
        w[d, 1] = int(np.rint(np.float32(c1 * np.float32(2048))))
        ofs[d] = s
    return ofs, w


def cv2_resize_linear_u8(img: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(img, (width, height)) for uint8 [H, W, C] (INTER_LINEAR)."""
    H, W, C = img.shape
    xo, xw = resize_coeffs(W, width)
    yo, yw = resize_coeffs(H, height)
    x1 = np.minimum(xo + 1, W - 1)
    src = img.astype(np.int64)
    hz = src[:, xo, :] * xw[None, :, 0, None] + src[:, x1, :] * xw[None, :, 1, None]   # [H, width, C]
    y1 = np.minimum(yo + 1, H - 1)
    S0, S1 = hz[yo], hz[y1]
    b0, b1 = yw[:, 0, None, None], yw[:, 1, None, None]
    v = (((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def cv2_bgr2gray_u8(img: np.ndarray) -> np.ndarray:
    b, g, r = (img[..., i].astype(np.int64) for i in range(3))
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def sls_image(bgr: np.ndarray, width: int = 128, height: int = 128) -> np.ndarray:
    """imread(BGR) -> resize -> BGR2GRAY -> /255.0, as the float32 the model is fed."""
    return (cv2_bgr2gray_u8(cv2_resize_linear_u8(bgr, width, height)) / 255.0).astype(np.float32)

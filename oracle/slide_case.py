"""Seeded synthetic slide and decoded outputs for the whole-slide inference parity tests -- TEST INFRASTRUCTURE
ONLY.  The slide has the geometry test.py:138-155 assumes (3092 x 2056 RGB); content: smooth per-channel
gradients + blobs + noise, uint8.  decoded(T, K): a (10, T, K) Wrapper-format stack (scores uniform in [0,1),
integer inds/ys/xs on the 128 map, axes, halo > minl, offsets in [0,4))."""
import numpy as np

SLIDE_H, SLIDE_W = 2056, 3092


def slide(seed=11, H=SLIDE_H, W=SLIDE_W):
    rs = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.zeros((H, W, 3), np.float32)
    for c in range(3):
        img[:, :, c] = 60 + 40 * np.sin(xx / (90 + 17 * c)) * np.cos(yy / (70 + 11 * c))
    for _ in range(200):
        cy, cx, r = rs.uniform(0, H), rs.uniform(0, W), rs.uniform(4, 20)
        y0, y1, x0, x1 = int(max(0, cy - 3 * r)), int(min(H, cy + 3 * r)), int(max(0, cx - 3 * r)), int(min(W, cx + 3 * r))
        g = np.exp(-((yy[y0:y1, x0:x1] - cy) ** 2 + (xx[y0:y1, x0:x1] - cx) ** 2) / (2 * r * r))
        img[y0:y1, x0:x1, :] += (120 * g)[:, :, None] * rs.uniform(0.5, 1, 3)[None, None, :]
    img += rs.normal(0, 6, img.shape)
    return np.clip(np.round(img), 0, 255).astype(np.uint8)


def decoded(T, K=100, seed=12):
    rs = np.random.RandomState(seed)
    ys = rs.randint(0, 128, (T, K))
    xs = rs.randint(0, 128, (T, K))
    minl = rs.uniform(0.5, 3, (T, K))
    rows = [rs.uniform(0, 1, (T, K)), ys * 128 + xs, ys, xs, rs.uniform(-6, 6, (T, K)), rs.uniform(-6, 6, (T, K)),
            minl, minl + rs.uniform(0, 4, (T, K)), rs.uniform(0, 4, (T, K)), rs.uniform(0, 4, (T, K))]
    return np.stack(rows).astype(np.float32)


def geometry(H, W, tile=512, pad=64):
    """test.py:41-54."""
    step = tile - 2 * pad
    ch, cv = -(-(W - 2 * pad) // step), -(-(H - 2 * pad) // step)
    rw, rh = step * ch + 2 * pad, step * cv + 2 * pad
    rw += (rw - W) % 2
    rh += (rh - H) % 2
    return dict(clipH=ch, clipV=cv, resizeW=rw, resizeH=rh, padLR=(rw - W) // 2, padTB=(rh - H) // 2)


def clip(img, g, i, j, tile=512, step=384):
    """Clip (i, j) of test.py:19-87 restated in numpy float64: greyscale, reflect padding, the opencv column
    fix-up, per-clip normalisation, float32."""
    grey = np.round(0.1140 * img[:, :, 0] + 0.5870 * img[:, :, 1] + 0.2989 * img[:, :, 2])
    pad = np.pad(grey, ((g["padTB"], g["padTB"]), (g["padLR"], g["padLR"])), mode="reflect")
    for x in range(0, 64):
        pad[:, x] = pad[:, 127 - x]
    for x in range(3136, 3200):
        pad[:, x] = pad[:, 6271 - x]
    t = pad[j * step:j * step + tile, i * step:i * step + tile]
    m = t.mean()
    return ((t - m) / np.sqrt(((t - m) ** 2).mean())).astype(np.float32)


def detections(dec, g, step=384, thr=0.3):
    """test.py:104-135 restated: [x, y, ratio] for every slot with score > thr, tile-major."""
    out = []
    T = dec.shape[1]
    for t in range(T):
        i, j = t // g["clipV"], t % g["clipV"]
        for k in range(dec.shape[2]):
            if dec[0, t, k] > np.float32(thr):
                minl, halo = float(dec[6, t, k]) * 4, float(dec[7, t, k]) * 4
                out.append([int(i * step - g["padLR"] + float(dec[3, t, k]) * 4 + float(dec[8, t, k])),
                            int(j * step - g["padTB"] + float(dec[2, t, k]) * 4 + float(dec[9, t, k])),
                            (halo - minl) / (2 * minl)])
    return np.array(out, np.float64).reshape(-1, 3)

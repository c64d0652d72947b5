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

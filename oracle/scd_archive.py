"""Seeded synthetic `.d` archives for the dataset-format parity tests -- TEST INFRASTRUCTURE ONLY.

The canonical archive holds FSI x ARGUM x CLIP = 49,920 tiles (datasets/scds/scdx16p100.py:143-156 index
that many), which the reference's loader needs to run at all; tiles here are tiny (8 x 8 float32) so the
whole archive is ~25 MB.  Objects: 0-4 per tile (some empty), fractional centres in [0,128) (exercising the
reference's int() truncation), the object-row layout of scdx16p100.py:380 [ctx, cty, offx, offy, majx, majy,
minl, halo].  Written through the product's writer (trainer/dataset/scdx16p100.writeArchive), whose layout
is checked against the reference's reader by tests/golden/make_golden_scd.py.
"""
import numpy as np

CANONICAL = 130 * 16 * 24


def archive_content(seed=2024, count=CANONICAL, size=8):
    rs = np.random.RandomState(seed)
    names = ["%d.%d" % (i // 384 + 1, i % 384 + 1) for i in range(count)]
    samples = rs.uniform(0, 255, (count, size, size)).astype(np.float32)
    nobj = rs.randint(0, 5, count)
    locs = []
    for n in nobj:
        l = np.zeros((n, 8), np.float32)
        l[:, 0:2] = rs.uniform(0, 128, (n, 2))
        l[:, 2:4] = rs.uniform(0, 4, (n, 2))
        length, ang = rs.uniform(2, 6, n), rs.uniform(0, np.pi, n)
        l[:, 4], l[:, 5] = length * np.cos(ang), length * np.sin(ang)
        l[:, 6] = rs.uniform(1, 3, n)
        l[:, 7] = l[:, 6] + rs.uniform(0, 4, n)
        locs.append(l)
    return names, list(samples), locs


def write(path, seed=2024, count=CANONICAL, size=8):
    from trainer.dataset.scdx16p100 import writeArchive
    names, samples, locs = archive_content(seed, count, size)
    writeArchive(path, names, samples, locs)
    return names, samples, locs

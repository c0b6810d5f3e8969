"""Datasets and cross-validation splits.

* ``make_cifar_like``  -- synthetic CIFAR-10-shaped data (32x32x3, 10
  classes) with *learnable* class structure (stroke glyphs + colour,
  translation, clutter and noise nuisances), the protocol fixed in
  BASELINE.md (there is no network, so real CIFAR-10 cannot be fetched).
* ``make_mnist_like``  -- same idea at 28x28x1 (reference driver config,
  tests/test_mnist.py:17-34, whose MNIST download is dead).
* ``load_iris_xy`` / ``load_wine_quality`` -- tabular fixtures for the GBDT
  species (BASELINE cfg 1; reference tests/test_wine-quality.py:15-19).
* ``stratified_kfold`` / ``kfold`` -- deterministic fold builders (the
  reference uses an unseeded ``StratifiedKFold(shuffle=True)``,
  gentun/models/keras_models.py:132; xgboost's ``cv`` uses seed 0).
"""

import os

import numpy as np


def _smooth_field(rng, h, w, c, scale):
    """Low-frequency random pattern in [-1, 1] (sum of a few 2-D cosines)."""
    yy, xx = np.meshgrid(np.linspace(0, 1, h, dtype=np.float32), np.linspace(0, 1, w, dtype=np.float32),
                         indexing="ij")
    out = np.zeros((h, w, c), np.float32)
    for ch in range(c):
        for _ in range(4):
            fy, fx = rng.uniform(0.5, scale, size=2)
            ph = rng.uniform(0, 2 * np.pi, size=2)
            out[:, :, ch] += np.cos(2 * np.pi * fy * yy + ph[0]) * np.cos(2 * np.pi * fx * xx + ph[1])
    out /= np.abs(out).max() + 1e-6
    return out


def _glyph(rng, size, strokes, width):
    """A random 'character': ``strokes`` anti-aliased line segments on a dark
    ``size`` x ``size`` canvas (values in [0, 1])."""
    yy, xx = np.meshgrid(np.arange(size, dtype=np.float32), np.arange(size, dtype=np.float32), indexing="ij")
    img = np.zeros((size, size), np.float32)
    lo, hi = 0.2 * size, 0.8 * size
    pts = rng.uniform(lo, hi, size=(strokes + 1, 2)).astype(np.float32)
    for k in range(strokes):
        # consecutive strokes share an end point (a pen trace), every other one restarts
        a = pts[k] if k % 2 == 0 else rng.uniform(lo, hi, size=2).astype(np.float32)
        b = pts[k + 1]
        d = b - a
        t = np.clip(((yy - a[0]) * d[0] + (xx - a[1]) * d[1]) / max(float(d @ d), 1e-6), 0.0, 1.0)
        dist = np.hypot(yy - (a[0] + t * d[0]), xx - (a[1] + t * d[1]))
        img = np.maximum(img, np.clip(1.0 - (dist - width) / 1.2, 0.0, 1.0))
    return img


def make_glyph_classification(n=10000, shape=(32, 32, 3), classes=10, seed=0, noise=0.5, shift=4, clutter=0.6,
                              dtype=np.float32):
    """Synthetic 'coloured glyph' images: every class owns a random stroke
    glyph (4 pen strokes); a sample is its class glyph translated by up to
    ``shift`` pixels, in a random stroke colour over a random dark background
    gradient, overlaid with a random other class's glyph at up to ``clutter``
    intensity and with Gaussian noise. High-contrast, edge-dominated content
    with the first-order statistics of natural image datasets scaled to [0,1]
    (a plain 12-conv ReLU stack trains on it, as on MNIST; smooth low-frequency
    synthetic data makes such stacks collapse at lr 1e-3)."""
    rng = np.random.default_rng(seed)
    h, w, c = shape
    size = max(h, w) + 2 * shift
    glyphs = np.stack([_glyph(rng, size, 4, 0.9 + 0.5 * rng.uniform()) for _ in range(classes)])
    labels = np.arange(n) % classes
    rng.shuffle(labels)
    dy = rng.integers(0, 2 * shift + 1, size=n)
    dx = rng.integers(0, 2 * shift + 1, size=n)
    ody = rng.integers(0, 2 * shift + 1, size=n)
    odx = rng.integers(0, 2 * shift + 1, size=n)
    other = (labels + rng.integers(1, classes, size=n)) % classes
    alpha = rng.uniform(0.0, clutter, size=n).astype(np.float32)
    color = rng.uniform(0.45, 1.0, size=(n, c)).astype(np.float32)
    ocolor = rng.uniform(0.2, 1.0, size=(n, c)).astype(np.float32)
    bg0 = rng.uniform(0.0, 0.25, size=(n, c)).astype(np.float32)
    bgslope = rng.uniform(-0.15, 0.15, size=(n, 2, c)).astype(np.float32)
    ramp_y = np.linspace(-0.5, 0.5, h, dtype=np.float32)[:, None, None]
    ramp_x = np.linspace(-0.5, 0.5, w, dtype=np.float32)[None, :, None]
    x = np.empty((n, h, w, c), np.float32)
    for i in range(n):
        g = glyphs[labels[i], dy[i]:dy[i] + h, dx[i]:dx[i] + w][:, :, None]
        o = glyphs[other[i], ody[i]:ody[i] + h, odx[i]:odx[i] + w][:, :, None]
        bg = bg0[i] + ramp_y * bgslope[i, 0] + ramp_x * bgslope[i, 1]
        img = bg * (1.0 - g) + color[i] * g
        x[i] = img * (1.0 - alpha[i] * o) + alpha[i] * ocolor[i] * o
    x += noise * 0.25 * rng.standard_normal(size=x.shape).astype(np.float32)
    np.clip(x, 0.0, 1.0, out=x)
    y = np.zeros((n, classes), np.float32)
    y[np.arange(n), labels] = 1.0
    return x.astype(dtype), y


def _stroke(rng, size, width, lo=0.15, hi=0.85):
    """One anti-aliased line segment in [0, 1] on a ``size`` x ``size`` canvas."""
    yy, xx = np.meshgrid(np.arange(size, dtype=np.float32), np.arange(size, dtype=np.float32), indexing="ij")
    a, b = rng.uniform(lo * size, hi * size, size=(2, 2)).astype(np.float32)
    d = b - a
    t = np.clip(((yy - a[0]) * d[0] + (xx - a[1]) * d[1]) / max(float(d @ d), 1e-6), 0.0, 1.0)
    dist = np.hypot(yy - (a[0] + t * d[0]), xx - (a[1] + t * d[1]))
    return np.clip(1.0 - (dist - width) / 1.2, 0.0, 1.0)


def make_parts_classification(n=10000, shape=(32, 32, 3), classes=10, seed=0, parts=8, per_class=3,
                              distractors=2, distract=(0.5, 1.0), same_color=False, noise=0.8, shift=4,
                              dtype=np.float32):
    """Compositional synthetic images: a pool of ``parts`` stroke primitives,
    every class the union of ``per_class`` of them (distinct combinations, so
    classes share strokes), a sample its class glyph translated by up to
    ``shift`` pixels plus ``distractors`` random single primitives of the
    pool at intensity ``distract`` (in their own colours), over a random
    background gradient, with Gaussian noise.

    Telling classes apart means recognising a CONJUNCTION of strokes among
    extra strokes from the same vocabulary: a sample with its class strokes
    plus a distractor also contains most of another class's strokes. Unlike
    :func:`make_glyph_classification` (one unique glyph per class; every
    architecture of the S=(3,5) space reaches ~0.99), accuracy here depends on
    the network: the bench data of BASELINE cfg 2-4 (``make_cifar_like``)."""
    rng = np.random.default_rng(seed)
    h, w, c = shape
    size = max(h, w) + 2 * shift
    prims = np.stack([_stroke(rng, size, 0.8 + 0.6 * rng.uniform()) for _ in range(parts)])
    combos, seen = [], set()
    while len(combos) < classes:
        k = tuple(sorted(rng.choice(parts, size=per_class, replace=False).tolist()))
        if k not in seen:
            seen.add(k)
            combos.append(k)
    glyphs = np.stack([prims[list(k)].max(0) for k in combos])
    labels = np.arange(n) % classes
    rng.shuffle(labels)
    dy = rng.integers(0, 2 * shift + 1, size=n)
    dx = rng.integers(0, 2 * shift + 1, size=n)
    color = rng.uniform(0.45, 1.0, size=(n, c)).astype(np.float32)
    bg0 = rng.uniform(0.0, 0.25, size=(n, c)).astype(np.float32)
    bgslope = rng.uniform(-0.15, 0.15, size=(n, 2, c)).astype(np.float32)
    ramp_y = np.linspace(-0.5, 0.5, h, dtype=np.float32)[:, None, None]
    ramp_x = np.linspace(-0.5, 0.5, w, dtype=np.float32)[None, :, None]
    dpart = rng.integers(0, parts, size=(n, distractors))
    dalpha = rng.uniform(distract[0], distract[1], size=(n, distractors)).astype(np.float32)
    dcolor = rng.uniform(0.3, 1.0, size=(n, distractors, c)).astype(np.float32)
    if same_color:                   # distractor strokes in the class glyph's colour: only shape tells them apart
        dcolor[:] = color[:, None, :]
    ddy = rng.integers(0, 2 * shift + 1, size=(n, distractors))
    ddx = rng.integers(0, 2 * shift + 1, size=(n, distractors))
    x = np.empty((n, h, w, c), np.float32)
    for i in range(n):
        g = glyphs[labels[i], dy[i]:dy[i] + h, dx[i]:dx[i] + w][:, :, None]
        img = (bg0[i] + ramp_y * bgslope[i, 0] + ramp_x * bgslope[i, 1]) * (1.0 - g) + color[i] * g
        for j in range(distractors):
            o = prims[dpart[i, j], ddy[i, j]:ddy[i, j] + h, ddx[i, j]:ddx[i, j] + w][:, :, None] * dalpha[i, j]
            img = img * (1.0 - o) + dcolor[i, j] * o
        x[i] = img
    x += noise * 0.25 * rng.standard_normal(size=x.shape).astype(np.float32)
    np.clip(x, 0.0, 1.0, out=x)
    y = np.zeros((n, classes), np.float32)
    y[np.arange(n), labels] = 1.0
    return x.astype(dtype), y


def make_relation_classification(n=10000, shape=(32, 32, 3), classes=10, seed=0, ptypes=5, psize=9, dist=(9, 13),
                                 distractors=2, noise=1.0, dtype=np.float32):
    """Relational synthetic images: ``ptypes`` small stroke parts
    (``psize`` x ``psize``); a class is an ordered PAIR of part types at a
    relative DIRECTION (right / below / left / above of each other, ``dist``
    pixels apart, +-1 jitter), classes chosen so that they share part types
    and directions. A sample places its pair anywhere in the image, adds
    ``distractors`` random parts elsewhere, all in one random colour, over a
    random background gradient, with Gaussian noise.

    The label is a relation between two parts ~11 pixels apart anywhere in the
    image: a network must see both parts in one receptive field, so deeper /
    wider DAG stages should beat shallow ones, and the distractors keep the
    part inventory alone from answering."""
    rng = np.random.default_rng(seed)
    h, w, c = shape
    parts = []
    for _ in range(ptypes):
        img = np.zeros((psize, psize), np.float32)
        for _ in range(2):
            img = np.maximum(img, _stroke(rng, psize, 0.5 + 0.4 * rng.uniform(), lo=0.05, hi=0.95))
        parts.append(img)
    parts = np.stack(parts)
    dirs = [(0, 1), (1, 0), (0, -1), (-1, 0)]
    combos, seen = [], set()
    while len(combos) < classes:
        a, b = rng.choice(ptypes, size=2, replace=True)
        d = int(rng.integers(0, 4))
        key = (int(a), int(b), d)
        mirror = (int(b), int(a), (d + 2) % 4)            # the same picture as another class
        if key not in seen and mirror not in seen:
            seen.add(key)
            combos.append(key)
    labels = np.arange(n) % classes
    rng.shuffle(labels)
    color = rng.uniform(0.45, 1.0, size=(n, c)).astype(np.float32)
    bg0 = rng.uniform(0.0, 0.25, size=(n, c)).astype(np.float32)
    bgslope = rng.uniform(-0.15, 0.15, size=(n, 2, c)).astype(np.float32)
    ramp_y = np.linspace(-0.5, 0.5, h, dtype=np.float32)[:, None, None]
    ramp_x = np.linspace(-0.5, 0.5, w, dtype=np.float32)[None, :, None]
    x = np.empty((n, h, w, c), np.float32)
    for i in range(n):
        a, b, d = combos[labels[i]]
        r = int(rng.integers(dist[0], dist[1] + 1))
        dy, dx = dirs[d][0] * r + int(rng.integers(-1, 2)), dirs[d][1] * r + int(rng.integers(-1, 2))
        # anchor of part a so that both parts are inside the image
        y0lo, y0hi = max(0, -dy), min(h - psize, h - psize - dy)
        x0lo, x0hi = max(0, -dx), min(w - psize, w - psize - dx)
        y0, x0 = int(rng.integers(y0lo, y0hi + 1)), int(rng.integers(x0lo, x0hi + 1))
        g = np.zeros((h, w), np.float32)
        g[y0:y0 + psize, x0:x0 + psize] = np.maximum(g[y0:y0 + psize, x0:x0 + psize], parts[a])
        g[y0 + dy:y0 + dy + psize, x0 + dx:x0 + dx + psize] = np.maximum(
            g[y0 + dy:y0 + dy + psize, x0 + dx:x0 + dx + psize], parts[b])
        for _ in range(distractors):
            k = int(rng.integers(0, ptypes))
            yy, xx = int(rng.integers(0, h - psize + 1)), int(rng.integers(0, w - psize + 1))
            g[yy:yy + psize, xx:xx + psize] = np.maximum(g[yy:yy + psize, xx:xx + psize], parts[k])
        gg = g[:, :, None]
        x[i] = (bg0[i] + ramp_y * bgslope[i, 0] + ramp_x * bgslope[i, 1]) * (1.0 - gg) + color[i] * gg
    x += noise * 0.25 * rng.standard_normal(size=x.shape).astype(np.float32)
    np.clip(x, 0.0, 1.0, out=x)
    y = np.zeros((n, classes), np.float32)
    y[np.arange(n), labels] = 1.0
    return x.astype(dtype), y


def make_compound_classification(n=10000, shape=(32, 32, 3), classes=10, seed=0, psize=11, msize=5, dist=(9, 12),
                                 distractors=1, noise=1.0, dtype=np.float32):
    """Two-level synthetic images: ``classes // 2`` glyph types (random
    2-stroke parts, ``psize`` pixels) times a SIDE -- a small marker
    (``msize``) sits left or right of the glyph, ``dist`` pixels apart
    (+-2 vertical jitter). Class = (glyph type, side). Placement is random, one
    distractor stroke is added elsewhere, colours / background / noise as in
    :func:`make_glyph_classification`.

    The glyph half of the label is easy (every architecture learns it: no
    collapse to chance, unlike a purely relational task); the side half needs
    the glyph and the marker in one receptive field ~12 pixels wide, which is
    what deeper DAG stages buy. So candidates spread between ~0.5 (glyph only)
    and ~1.0 (glyph and side) by architecture."""
    rng = np.random.default_rng(seed)
    h, w, c = shape
    ntype = classes // 2
    glyphs = []
    for _ in range(ntype):
        img = np.zeros((psize, psize), np.float32)
        for _ in range(2):
            img = np.maximum(img, _stroke(rng, psize, 0.6 + 0.4 * rng.uniform(), lo=0.05, hi=0.95))
        glyphs.append(img)
    yy, xx = np.meshgrid(np.arange(msize, dtype=np.float32), np.arange(msize, dtype=np.float32), indexing="ij")
    r = (msize - 1) / 2.0
    marker = np.clip(1.0 - (np.hypot(yy - r, xx - r) - 0.35 * msize) / 1.0, 0.0, 1.0)      # a filled dot
    labels = np.arange(n) % (2 * ntype)
    rng.shuffle(labels)
    color = rng.uniform(0.45, 1.0, size=(n, c)).astype(np.float32)
    bg0 = rng.uniform(0.0, 0.25, size=(n, c)).astype(np.float32)
    bgslope = rng.uniform(-0.15, 0.15, size=(n, 2, c)).astype(np.float32)
    ramp_y = np.linspace(-0.5, 0.5, h, dtype=np.float32)[:, None, None]
    ramp_x = np.linspace(-0.5, 0.5, w, dtype=np.float32)[None, :, None]
    mo = (psize - msize) // 2
    x = np.empty((n, h, w, c), np.float32)
    for i in range(n):
        t, side = labels[i] // 2, labels[i] % 2
        d = int(rng.integers(dist[0], dist[1] + 1)) * (1 if side else -1)
        jy = int(rng.integers(-2, 3))
        # glyph box at (y0, x0); marker box at (y0 + mo + jy, x0 + mo + d), both inside the image
        xlo, xhi = max(0, -(mo + d)), min(w - psize, w - msize - mo - d)
        ylo, yhi = max(0, -(mo + jy)), min(h - psize, h - msize - mo - jy)
        y0, x0 = int(rng.integers(ylo, yhi + 1)), int(rng.integers(xlo, xhi + 1))
        g = np.zeros((h, w), np.float32)
        g[y0:y0 + psize, x0:x0 + psize] = glyphs[t]
        my, mx = y0 + mo + jy, x0 + mo + d
        g[my:my + msize, mx:mx + msize] = np.maximum(g[my:my + msize, mx:mx + msize], marker)
        for _ in range(distractors):
            s = _stroke(rng, 9, 0.6, lo=0.1, hi=0.9)
            yy0, xx0 = int(rng.integers(0, h - 8)), int(rng.integers(0, w - 8))
            g[yy0:yy0 + 9, xx0:xx0 + 9] = np.maximum(g[yy0:yy0 + 9, xx0:xx0 + 9], 0.8 * s)
        gg = g[:, :, None]
        x[i] = (bg0[i] + ramp_y * bgslope[i, 0] + ramp_x * bgslope[i, 1]) * (1.0 - gg) + color[i] * gg
    x += noise * 0.25 * rng.standard_normal(size=x.shape).astype(np.float32)
    np.clip(x, 0.0, 1.0, out=x)
    y = np.zeros((n, 2 * ntype), np.float32)
    y[np.arange(n), labels] = 1.0
    return x.astype(dtype), y


def make_variant_classification(n=10000, shape=(32, 32, 3), classes=10, seed=0, noise=1.0, shift=5, clutter=0.8,
                                tick=6, tick_width=0.7, label_noise=0.0, dtype=np.float32):
    """Coarse + fine classes: ``classes // 2`` base glyphs (the 4-stroke
    glyphs of :func:`make_glyph_classification`, whose strong, image-wide
    signal every architecture picks up early -- no extra collapse to chance),
    each in two VARIANTS that carry a short ``tick``-pixel stroke at one of two
    glyph-relative places (variant A vs B). A sample is translated, coloured,
    cluttered by another base glyph (without tick) and noised as in the glyph
    set. The base glyph answers half of the label; the variant needs the small
    tick localised relative to its glyph under clutter and noise -- the part
    that should separate architectures (BASELINE cfg 2-4 bench data,
    ``make_cifar_like``)."""
    rng = np.random.default_rng(seed)
    h, w, c = shape
    size = max(h, w) + 2 * shift
    nb = classes // 2
    base = np.stack([_glyph(rng, size, 4, 0.9 + 0.5 * rng.uniform()) for _ in range(nb)])
    variants = []
    for k in range(nb):
        for _ in range(2):
            t = np.zeros((size, size), np.float32)
            cy, cx = rng.uniform(0.3 * size, 0.7 * size, size=2)
            ang = rng.uniform(0, np.pi)
            a = np.array([cy - 0.5 * tick * np.sin(ang), cx - 0.5 * tick * np.cos(ang)], np.float32)
            b = np.array([cy + 0.5 * tick * np.sin(ang), cx + 0.5 * tick * np.cos(ang)], np.float32)
            yy, xx = np.meshgrid(np.arange(size, dtype=np.float32), np.arange(size, dtype=np.float32), indexing="ij")
            d = b - a
            tt = np.clip(((yy - a[0]) * d[0] + (xx - a[1]) * d[1]) / max(float(d @ d), 1e-6), 0.0, 1.0)
            dist = np.hypot(yy - (a[0] + tt * d[0]), xx - (a[1] + tt * d[1]))
            t = np.clip(1.0 - (dist - tick_width) / 1.2, 0.0, 1.0)
            variants.append(np.maximum(base[k], t))
    glyphs = np.stack(variants)                          # class k*2 + v
    labels = np.arange(n) % (2 * nb)
    rng.shuffle(labels)
    dy = rng.integers(0, 2 * shift + 1, size=n)
    dx = rng.integers(0, 2 * shift + 1, size=n)
    ody = rng.integers(0, 2 * shift + 1, size=n)
    odx = rng.integers(0, 2 * shift + 1, size=n)
    other = (labels // 2 + rng.integers(1, nb, size=n)) % nb
    alpha = rng.uniform(0.0, clutter, size=n).astype(np.float32)
    color = rng.uniform(0.45, 1.0, size=(n, c)).astype(np.float32)
    ocolor = rng.uniform(0.2, 1.0, size=(n, c)).astype(np.float32)
    bg0 = rng.uniform(0.0, 0.25, size=(n, c)).astype(np.float32)
    bgslope = rng.uniform(-0.15, 0.15, size=(n, 2, c)).astype(np.float32)
    ramp_y = np.linspace(-0.5, 0.5, h, dtype=np.float32)[:, None, None]
    ramp_x = np.linspace(-0.5, 0.5, w, dtype=np.float32)[None, :, None]
    x = np.empty((n, h, w, c), np.float32)
    for i in range(n):
        g = glyphs[labels[i], dy[i]:dy[i] + h, dx[i]:dx[i] + w][:, :, None]
        o = base[other[i], ody[i]:ody[i] + h, odx[i]:odx[i] + w][:, :, None]
        bg = bg0[i] + ramp_y * bgslope[i, 0] + ramp_x * bgslope[i, 1]
        img = bg * (1.0 - g) + color[i] * g
        x[i] = img * (1.0 - alpha[i] * o) + alpha[i] * ocolor[i] * o
    x += noise * 0.25 * rng.standard_normal(size=x.shape).astype(np.float32)
    np.clip(x, 0.0, 1.0, out=x)
    if label_noise > 0:
        # a fraction of the labels names the OTHER variant of the same base glyph: the best achievable
        # accuracy is 1 - label_noise, and a network that memorises the flips validates lower
        flip = rng.uniform(size=n) < label_noise
        labels = np.where(flip, labels ^ 1, labels)
    y = np.zeros((n, 2 * nb), np.float32)
    y[np.arange(n), labels] = 1.0
    return x.astype(dtype), y


def make_image_classification(n=10000, shape=(32, 32, 3), classes=10, seed=0, noise=0.35, shift=3,
                              dtype=np.float32):
    """Synthetic image classification set: x in [0,1] NHWC, y one-hot.

    Each class owns a smooth template; a sample is its template, randomly
    translated by up to ``shift`` pixels, contrast/brightness jittered,
    mixed with a second class's template at low weight and with Gaussian
    noise. A small CNN reaches well above chance but not 100 %, so the GA
    has signal to optimise.
    """
    rng = np.random.default_rng(seed)
    h, w, c = shape
    templates = np.stack([_smooth_field(rng, h + 2 * shift, w + 2 * shift, c, 4.0) for _ in range(classes)])
    labels = np.arange(n) % classes
    rng.shuffle(labels)
    x = np.empty((n, h, w, c), np.float32)
    dy = rng.integers(0, 2 * shift + 1, size=n)
    dx = rng.integers(0, 2 * shift + 1, size=n)
    amp = rng.uniform(0.5, 1.0, size=n).astype(np.float32)
    bright = rng.uniform(-0.1, 0.1, size=n).astype(np.float32)
    other = rng.integers(0, classes, size=n)
    mix = rng.uniform(0.0, 0.45, size=n).astype(np.float32)
    for i in range(n):
        t = templates[labels[i], dy[i]:dy[i] + h, dx[i]:dx[i] + w]
        o = templates[other[i], dy[i]:dy[i] + h, dx[i]:dx[i] + w]
        x[i] = 0.5 + 0.25 * amp[i] * (t + mix[i] * o) + bright[i]
    x += noise * 0.25 * rng.standard_normal(size=x.shape).astype(np.float32)
    np.clip(x, 0.0, 1.0, out=x)
    y = np.zeros((n, classes), np.float32)
    y[np.arange(n), labels] = 1.0
    return x.astype(dtype), y


def make_cifar_like(n=10000, seed=0, noise=1.0, shift=5, clutter=0.8):
    """Bench dataset (BASELINE.json Genetic-CNN configs): 32x32x3 coloured
    glyphs, 10 classes. Noise / clutter are set so that every architecture of
    the S=(3,5) space -- including the 12-conv chains -- learns under the
    reference schedule, yet architectures still differ in validation score.
    (The smooth-template generator ``make_image_classification`` at high noise
    made every deep chain collapse to a constant softmax -- binary accuracy
    0.9 -- in both the HIP and the PyTorch executors.)"""
    return make_glyph_classification(n=n, shape=(32, 32, 3), classes=10, seed=seed, noise=noise, shift=shift,
                                     clutter=clutter)


def make_cifar_hard(n=10000, seed=0):
    """Discriminative bench dataset (round 3): :func:`make_variant_classification`
    with 30 % of the variant labels flipped and noise 0.7 -- five base glyphs x
    two tick variants. Measured on 12 random S=(3,5) candidates under the full
    reference protocol (profiles/dataset_spread_r3.txt): a learned fold scores
    0.61-0.66 (the flips cap it at 0.70; how much of them a network memorises
    depends on its architecture), 4 of 60 folds collapsed to chance -- unlike
    :func:`make_cifar_like`, where every learned fold saturates at 0.98-0.99 and
    only fold collapse separates candidates."""
    return make_variant_classification(n=n, shape=(32, 32, 3), classes=10, seed=seed, noise=0.7, label_noise=0.3)


def make_mnist_like(n=10000, seed=0, noise=1.0, shift=4, clutter=0.8):
    """28x28x1 glyphs (reference driver config, tests/test_mnist.py:17-34,
    whose MNIST download is dead)."""
    return make_glyph_classification(n=n, shape=(28, 28, 1), classes=10, seed=seed, noise=noise, shift=shift,
                                     clutter=clutter)


def load_iris_xy():
    """Iris (150x4, 3 classes) from scikit-learn's bundled copy."""
    from sklearn.datasets import load_iris
    d = load_iris()
    return d.data.astype(np.float64), d.target.astype(np.float64)


def load_wine_quality(path=None):
    """White wine quality (4,898 x 11 -> quality). ``path`` defaults to the
    vendored copy of the public UCI fixture the reference ships
    (tests/data/winequality-white.csv, ';'-separated)."""
    import pandas as pd
    if path is None:
        here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        path = os.environ.get("GENTUN_WINE_CSV", os.path.join(here, "tests", "data", "winequality-white.csv"))
    df = pd.read_csv(path, sep=";")
    y = df.pop("quality").to_numpy(np.float64)
    return df.to_numpy(np.float64), y


def make_regression(n=100000, f=32, seed=0, noise=0.1):
    """Synthetic tabular regression with non-linear structure (GBDT bench)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, f)).astype(np.float32)
    y = (np.sin(x[:, 0]) + 0.5 * x[:, 1] * x[:, 2] + np.where(x[:, 3] > 0, 1.0, -0.5)
         + 0.25 * x[:, 4] ** 2 + noise * rng.standard_normal(n)).astype(np.float32)
    return x, y


# ---------------------------------------------------------------------------
# Cross-validation splits
# ---------------------------------------------------------------------------

def labels_from_onehot(y):
    y = np.asarray(y)
    if y.ndim == 2:
        return np.argmax(y, axis=1)
    return y.astype(np.int64)


def stratified_kfold(labels, nfold, seed=0):
    """Deterministic stratified shuffled k-fold.

    Returns a list of ``(train_idx, val_idx)`` int64 arrays. Per class the
    sample indices are shuffled with ``seed`` and dealt to folds in turn, so
    fold sizes differ by at most one per class (sklearn semantics).
    """
    labels = np.asarray(labels)
    n = labels.shape[0]
    rng = np.random.default_rng(seed)
    fold_of = np.empty(n, np.int64)
    offset = 0
    for cls in np.unique(labels):
        idx = np.flatnonzero(labels == cls)
        rng.shuffle(idx)
        fold_of[idx] = (np.arange(idx.size) + offset) % nfold
        offset += idx.size
    out = []
    for k in range(nfold):
        val = np.flatnonzero(fold_of == k)
        train = np.flatnonzero(fold_of != k)
        out.append((train, val))
    return out


def kfold(n, nfold, seed=0, shuffle=True):
    """Plain k-fold (xgboost ``cv`` default: shuffled, not stratified)."""
    idx = np.arange(n)
    if shuffle:
        np.random.default_rng(seed).shuffle(idx)
    parts = np.array_split(idx, nfold)
    out = []
    for k in range(nfold):
        val = np.sort(parts[k])
        train = np.sort(np.concatenate([parts[j] for j in range(nfold) if j != k]))
        out.append((train, val))
    return out

"""Draw a decoded Genetic-CNN plan as a graph image (``GeneticCnnModel.plot``).

The reference calls Keras' ``plot_model`` (gentun/models/keras_models.py:
41-44), which needs pydot + graphviz; neither is available here, so the
layered layout and the rasteriser are our own: nodes are placed by their
longest-path depth from the input, edges are straight lines with arrowheads,
and N-ary sums (Keras ``Add`` layers) are drawn as their own "add" nodes.

Output by file suffix: ``.png`` (the reference's format; pure-Python
encoder, built-in 5x7 bitmap font), ``.svg`` or ``.dot`` (Graphviz text).
"""

import struct
import zlib

import numpy as np

from ..models.genome import ConvSpec

# 5x7 bitmap glyphs: 7 rows of 5 bits (MSB = leftmost column)
_FONT = {
    'a': "00000 00000 01110 00001 01111 10001 01111", 'b': "10000 10000 11110 10001 10001 10001 11110",
    'c': "00000 00000 01110 10000 10000 10001 01110", 'd': "00001 00001 01111 10001 10001 10001 01111",
    'e': "00000 00000 01110 10001 11111 10000 01110", 'f': "00110 01001 01000 11100 01000 01000 01000",
    'g': "00000 01111 10001 10001 01111 00001 01110", 'h': "10000 10000 10110 11001 10001 10001 10001",
    'i': "00100 00000 01100 00100 00100 00100 01110", 'j': "00010 00000 00110 00010 00010 10010 01100",
    'k': "10000 10000 10010 10100 11000 10100 10010", 'l': "01100 00100 00100 00100 00100 00100 01110",
    'm': "00000 00000 11010 10101 10101 10001 10001", 'n': "00000 00000 10110 11001 10001 10001 10001",
    'o': "00000 00000 01110 10001 10001 10001 01110", 'p': "00000 11110 10001 10001 11110 10000 10000",
    'q': "00000 01111 10001 10001 01111 00001 00001", 'r': "00000 00000 10110 11001 10000 10000 10000",
    's': "00000 00000 01110 10000 01110 00001 11110", 't': "01000 01000 11100 01000 01000 01001 00110",
    'u': "00000 00000 10001 10001 10001 10011 01101", 'v': "00000 00000 10001 10001 10001 01010 00100",
    'w': "00000 00000 10001 10001 10101 10101 01010", 'x': "00000 00000 10001 01010 00100 01010 10001",
    'y': "00000 00000 10001 10001 01111 00001 01110", 'z': "00000 00000 11111 00010 00100 01000 11111",
    '0': "01110 10001 10011 10101 11001 10001 01110", '1': "00100 01100 00100 00100 00100 00100 01110",
    '2': "01110 10001 00001 00010 00100 01000 11111", '3': "11111 00010 00100 00010 00001 10001 01110",
    '4': "00010 00110 01010 10010 11111 00010 00010", '5': "11111 10000 11110 00001 00001 10001 01110",
    '6': "00110 01000 10000 11110 10001 10001 01110", '7': "11111 00001 00010 00100 01000 01000 01000",
    '8': "01110 10001 10001 01110 10001 10001 01110", '9': "01110 10001 10001 01111 00001 00010 01100",
    '_': "00000 00000 00000 00000 00000 00000 11111", '-': "00000 00000 00000 11111 00000 00000 00000",
    '>': "10000 01000 00100 00010 00100 01000 10000", '(': "00010 00100 01000 01000 01000 00100 00010",
    ')': "01000 00100 00010 00010 00010 00100 01000", '+': "00000 00100 00100 11111 00100 00100 00000",
    '.': "00000 00000 00000 00000 00000 01100 01100", ',': "00000 00000 00000 00000 01100 00100 01000",
    ' ': "00000 00000 00000 00000 00000 00000 00000", ':': "00000 01100 01100 00000 01100 01100 00000",
}
_GLYPHS = {ch: np.array([[c == '1' for c in row] for row in rows.split()], bool) for ch, rows in _FONT.items()}
_SCALE = 2                          # font pixels per glyph bit
_CW, _CH = 6 * _SCALE, 8 * _SCALE   # character cell


def graph_of(plan):
    """Nodes ``[(id, label)]`` and edges ``[(src, dst)]`` of a plan: conv,
    add (a sum of >1 tensors), pool, and the dense head."""
    nodes, edges = [("input", "input {}x{}x{}".format(*plan.input_shape))], []

    def source(srcs, name):
        if len(srcs) == 1:
            return srcs[0]
        add = name + "_add"
        nodes.append((add, "add"))
        edges.extend((s, add) for s in srcs)
        return add

    for st in plan.steps:
        if isinstance(st, ConvSpec):
            src = source(st.inputs, st.name)
            nodes.append((st.name, "{} conv{}x{} {}->{}".format(st.name, st.k[0], st.k[1], st.cin, st.cout)))
        else:
            src = source(st.srcs, st.name)
            nodes.append((st.name, "{} maxpool2x2".format(st.name)))
        edges.append((src, st.name))
    last = plan.steps[-1].name
    head = [("flatten", "flatten {}".format(plan.flatten)), ("dense1", "dense {} relu".format(plan.dense_units)),
            ("dropout", "dropout"), ("dense2", "dense {} softmax".format(plan.classes))]
    for nid, label in head:
        nodes.append((nid, label))
        edges.append((last, nid))
        last = nid
    return nodes, edges


def layout(nodes, edges):
    """``{id: (col, row)}``: row = longest-path depth, columns in order."""
    depth = {nodes[0][0]: 0}
    preds = {}
    for s, d in edges:
        preds.setdefault(d, []).append(s)
    for nid, _ in nodes[1:]:           # nodes are topologically ordered
        depth[nid] = 1 + max(depth[p] for p in preds[nid])
    rows = {}
    pos = {}
    for nid, _ in nodes:
        r = depth[nid]
        pos[nid] = (rows.get(r, 0), r)
        rows[r] = rows.get(r, 0) + 1
    return pos, rows


def to_dot(plan):
    nodes, edges = graph_of(plan)
    out = ["digraph GeneticCNN {", "  node [shape=box];"]
    out += ['  "{}" [label="{}"];'.format(n, l) for n, l in nodes]
    out += ['  "{}" -> "{}";'.format(s, d) for s, d in edges]
    return "\n".join(out + ["}"]) + "\n"


def _geometry(plan):
    nodes, edges = graph_of(plan)
    pos, rows = layout(nodes, edges)
    labels = dict(nodes)
    bw = max(len(l) for l in labels.values()) * _CW + 12
    bh, gx, gy = _CH + 10, 24, 26
    ncol = max(rows.values())
    width = ncol * (bw + gx) + gx
    height = len(rows) * (bh + gy) + gy
    boxes = {}
    for nid, (c, r) in pos.items():
        off = (ncol - rows[r]) * (bw + gx) // 2          # centre each row
        x0, y0 = gx + off + c * (bw + gx), gy + r * (bh + gy)
        boxes[nid] = (x0, y0, x0 + bw, y0 + bh)
    return nodes, edges, labels, boxes, width, height


def to_svg(plan):
    nodes, edges, labels, boxes, width, height = _geometry(plan)
    out = ['<svg xmlns="http://www.w3.org/2000/svg" width="{}" height="{}" font-family="monospace" '
           'font-size="12">'.format(width, height),
           '<defs><marker id="a" markerWidth="8" markerHeight="8" refX="8" refY="4" orient="auto">'
           '<path d="M0,0 L8,4 L0,8 z"/></marker></defs>', '<rect width="100%" height="100%" fill="white"/>']
    for s, d in edges:
        a, b = boxes[s], boxes[d]
        out.append('<line x1="{}" y1="{}" x2="{}" y2="{}" stroke="black" marker-end="url(#a)"/>'.format(
            (a[0] + a[2]) // 2, a[3], (b[0] + b[2]) // 2, b[1]))
    for nid, (x0, y0, x1, y1) in boxes.items():
        out.append('<rect x="{}" y="{}" width="{}" height="{}" fill="#eef" stroke="black"/>'.format(
            x0, y0, x1 - x0, y1 - y0))
        out.append('<text x="{}" y="{}">{}</text>'.format(x0 + 6, y1 - 8, labels[nid]))
    return "\n".join(out + ["</svg>"]) + "\n"


def _line(img, x0, y0, x1, y1):
    n = max(abs(x1 - x0), abs(y1 - y0), 1)
    xs = np.round(np.linspace(x0, x1, n + 1)).astype(int)
    ys = np.round(np.linspace(y0, y1, n + 1)).astype(int)
    ok = (xs >= 0) & (xs < img.shape[1]) & (ys >= 0) & (ys < img.shape[0])
    img[ys[ok], xs[ok]] = 0


def _text(img, x, y, s):
    for i, ch in enumerate(s.lower()):
        g = _GLYPHS.get(ch, _GLYPHS[' '])
        big = np.kron(g, np.ones((_SCALE, _SCALE), bool))
        ys, xs = np.nonzero(big)
        img[y + ys, x + i * _CW + xs] = 0


def to_png_array(plan):
    """Greyscale uint8 image (255 = white) of the plan's graph."""
    nodes, edges, labels, boxes, width, height = _geometry(plan)
    img = np.full((height, width), 255, np.uint8)
    for s, d in edges:
        a, b = boxes[s], boxes[d]
        xa, ya, xb, yb = (a[0] + a[2]) // 2, a[3], (b[0] + b[2]) // 2, b[1]
        _line(img, xa, ya, xb, yb)
        # arrowhead at the destination
        v = np.array([xb - xa, yb - ya], float)
        v /= max(1e-9, np.hypot(*v))
        for sgn in (1, -1):
            w = np.array([-v[1], v[0]]) * sgn
            tip = np.array([xb, yb]) - 7 * v + 4 * w
            _line(img, xb, yb, int(tip[0]), int(tip[1]))
    for nid, (x0, y0, x1, y1) in boxes.items():
        img[y0:y1 + 1, x0:x1 + 1] = 238
        img[y0, x0:x1 + 1] = img[y1, x0:x1 + 1] = 0
        img[y0:y1 + 1, x0] = img[y0:y1 + 1, x1] = 0
        _text(img, x0 + 6, y0 + 5, labels[nid])
    return img


def encode_png(img):
    """8-bit greyscale PNG bytes of a 2-D uint8 array (stdlib zlib only)."""
    h, w = img.shape
    raw = b"".join(b"\x00" + img[r].tobytes() for r in range(h))

    def chunk(kind, data):
        return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b""))


def plot_plan(plan, path):
    """Write the plan's graph to ``path`` (.png, .svg or .dot); returns path."""
    low = path.lower()
    if low.endswith(".svg"):
        data = to_svg(plan).encode()
    elif low.endswith(".dot"):
        data = to_dot(plan).encode()
    else:
        data = encode_png(to_png_array(plan))
    with open(path, "wb") as f:
        f.write(data)
    return path

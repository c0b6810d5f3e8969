"""Launch schedule of a population-batched Genetic-CNN train step.

Pure Python (no device work): from the decoded plans of every group (a group
= one cross-validation fold of one candidate) it derives the *superset*
network -- per stage an input conv, ``K`` DAG node convs, an output conv and
a 2x2 pool (gentun/models/keras_models.py:46-118) -- and, for every launch,
which groups take part and what each one does:

* forward conv: the input slots it sums (bit k = ``layer.slots[k]``);
* pool: whether it pools the stage's output conv (stage has a DAG) or its
  input conv;
* backward: per layer, the data-gradient's fan-out flags -- write or
  accumulate into each input slot's gradient, and whether this launch is the
  slot's LAST writer (its first consumer in forward order), which applies
  the slot's ReLU mask -- and the weight-gradient's input (one slot, or the
  input sum the forward wrote for N-ary groups).

:class:`gentun_amd.models.cnn_hip.HipPopJob` turns these records into device
tables (csrc/hip/cnn_args.h ``GroupRec``); ``tests/test_pop_schedule.py``
executes them on the CPU with plain PyTorch ops and compares every group's
weight gradients with autograd through that group's own plan.
"""

from .genome import decode_stage

# GroupRec.out_mask fields: bit k write slot k, bit ACC_SHIFT+k accumulate
# into it, bit MASK_SHIFT+k apply its ReLU mask
ACC_SHIFT, MASK_SHIFT = 8, 16


def stage_topology(bits, nodes):
    """``(active, in_sets, sinks)`` of one stage of one candidate.

    ``in_sets[j]``: input slot indices of node j (0 = the stage's input conv,
    i + 1 = node i), ``None`` for an isolated node; ``sinks``: nodes summed
    into the output conv. ``active`` is False for an all-zero stage (no DAG,
    keras_models.py:108)."""
    if not any(b == '1' for b in bits):
        return False, None, None
    preds, _succs, active, outputs = decode_stage(bits, nodes)
    in_sets = [None] * nodes
    for j in range(nodes):
        if active[j]:
            in_sets[j] = [0] if not preds[j] else [p + 1 for p in preds[j]]
    return True, in_sets, list(outputs)


def mask_of(slots):
    m = 0
    for k in slots:
        m |= 1 << k
    return m


def popcount(x):
    return bin(x).count("1")


class LayerSpec(object):
    """One superset conv layer ('in', 'node' j or 'out' of a stage)."""

    def __init__(self, name, kind, j, stage, H, W, cin, cout, k, slots, rows):
        self.name, self.kind, self.j, self.stage = name, kind, j, stage
        self.H, self.W = H, W
        self.cin, self.cout = cin, cout
        self.KH, self.KW = k
        self.slots = slots        # input slot names; bit k of a row's in_mask = slots[k]
        self.rows = rows          # [(group, in_mask)], ascending group
        # groups summing > 1 input: the forward writes the sum to "<name>_xin"
        # and the wgrad reads that one slot
        self.xin = name + "_xin" if any(popcount(im) > 1 for _, im in rows) else None


class StageSpec(object):
    def __init__(self, s, H, W, x_slot, prefix, active):
        self.s, self.H, self.W = s, H, W
        self.x_slot = x_slot                  # stage input: "input" (the dataset) or the previous pool
        self.inp, self.out, self.pool = prefix + "_in", prefix + "_out", prefix + "_pool"
        self.active = active                  # per group: the stage has a DAG
        self.layers = []
        self.has_out = False                  # some group has the output conv


class PopulationSchedule(object):
    """Superset layers and per-launch group records for ``plans`` (one plan
    per group; the plans of one job share the search space, only genes
    differ)."""

    def __init__(self, plans, hw=None):
        """``hw``: the (H, W) the layers run at when it differs from the plans' input
        shape (a zero-padded image, cnn_kernels.padded_hw); stages also record
        their real extent (``Hr`` / ``Wr``)."""
        self.Q = len(plans)
        p0 = plans[0]
        for p in plans:
            if (p.nodes, p.input_shape, p.kernels_per_layer, p.kernel_sizes, p.dense_units, p.classes) != \
                    (p0.nodes, p0.input_shape, p0.kernels_per_layer, p0.kernel_sizes, p0.dense_units, p0.classes):
                raise ValueError("population members must share the search space (only genes may differ)")
        self.plan = p0
        topo = {}
        per_group = []
        for p in plans:
            key = tuple(sorted(p.genes.items()))
            if key not in topo:
                topo[key] = [stage_topology(p.genes["S_{}".format(s + 1)], p.nodes[s])
                             for s in range(len(p.kernels_per_layer))]
            per_group.append(topo[key])
        h0r, w0r, c0 = p0.input_shape
        h0, w0 = hw or (h0r, w0r)
        self.stages, self.layers = [], []
        cin, x_slot = c0, "input"
        for s, cout in enumerate(p0.kernels_per_layer):
            H, W = h0 >> s, w0 >> s
            Kn = p0.nodes[s]
            k = tuple(p0.kernel_sizes[s])
            if k[0] % 2 == 0 or k[1] % 2 == 0:
                raise ValueError("only odd kernel sizes are supported ('same' padding)")
            pre = "s{}".format(s + 1)
            st = StageSpec(s, H, W, x_slot, pre, [per_group[q][s][0] for q in range(self.Q)])
            st.Hr, st.Wr = h0r >> s, w0r >> s

            def add(name, kind, j, cin_, k_, slots, rows):
                if rows:
                    L = LayerSpec(name, kind, j, s, H, W, cin_, cout, k_, slots, rows)
                    L.Hr, L.Wr = st.Hr, st.Wr
                    st.layers.append(L)
                    self.layers.append(L)

            add(st.inp, "in", -1, cin, k, [x_slot], [(q, 1) for q in range(self.Q)])
            node_slots = [st.inp] + ["{}_n{}".format(pre, i) for i in range(Kn)]
            for j in range(Kn):
                rows = [(q, mask_of(per_group[q][s][1][j])) for q in range(self.Q)
                        if per_group[q][s][0] and per_group[q][s][1][j] is not None]
                add("{}_n{}".format(pre, j), "node", j, cout, (3, 3), node_slots[:j + 1], rows)
            rows = [(q, mask_of(per_group[q][s][2])) for q in range(self.Q) if per_group[q][s][0]]
            add(st.out, "out", -1, cout, (3, 3), node_slots[1:], rows)
            st.has_out = bool(rows)
            self.stages.append(st)
            x_slot, cin = st.pool, cout
        self.last = x_slot
        self.layer_names = set(L.name for L in self.layers)

    # -------------------------------------------------------------- forward
    def pool_source(self, st):
        """Per group: 1 = pool the stage's output conv, 0 = its input conv."""
        return [1 if a else 0 for a in st.active]

    def pool_x1(self, st):
        """Slot read by the pool for groups with a DAG (the input conv if no
        group of the job has one: then no group selects it)."""
        return st.out if st.has_out else st.inp

    # ------------------------------------------------------------- backward
    def backward(self):
        """Backward launch sequence, in issue order:

        * ``("pool_bwd", stage)``;
        * ``("wgrad", layer, rows)``, rows ``(group, in_mask)`` over the
          wgrad's slots (``layer.slots`` plus the input-sum slot at bit
          ``len(layer.slots)``);
        * ``("dgrad", layer, rows)`` (not for the first layer: the dataset
          has no gradient), rows ``(group, out_flags)``: bit k = write slot
          k's gradient, bit ACC_SHIFT+k = accumulate into it, bit
          MASK_SHIFT+k = apply slot k's ReLU mask (this launch is the slot's
          last writer, i.e. its first consumer in forward order)."""
        first_consumer = {}
        for L in self.layers:
            for q, im in L.rows:
                for k, n in enumerate(L.slots):
                    if (im >> k) & 1:
                        first_consumer.setdefault((q, n), L.name)
        written = set()
        seq = []
        for st in reversed(self.stages):
            seq.append(("pool_bwd", st))
            for q in range(self.Q):
                written.add((q, st.out if st.active[q] else st.inp))
            for L in reversed(st.layers):
                xbit = 1 << len(L.slots)
                seq.append(("wgrad", L, [(q, xbit if popcount(im) > 1 else im) for q, im in L.rows]))
                if L.slots == ["input"]:
                    continue
                rows = []
                for q, im in L.rows:
                    of = 0
                    for k, n in enumerate(L.slots):
                        if not (im >> k) & 1:
                            continue
                        of |= 1 << k
                        if (q, n) in written:
                            of |= 1 << (ACC_SHIFT + k)
                        # ReLU masks: conv outputs only (a pool output's comes
                        # through pool_bwd), applied by the slot's last writer
                        if L.kind != "in" and n in self.layer_names and first_consumer.get((q, n)) == L.name:
                            of |= 1 << (MASK_SHIFT + k)
                        written.add((q, n))
                    rows.append((q, of))
                seq.append(("dgrad", L, rows))
        return seq

"""Genetic-CNN genome decoding and cost model.

Decoding rules reproduce gentun/models/keras_models.py:46-118 exactly
(SURVEY.md §2.2 "Genetic-CNN decoding", test vectors in Appendix A.1):

* stage ``s`` bits split into consecutive chunks of sizes 1, 2, ..., K-1;
  chunk ``j`` lists which of nodes ``0..j`` feed node ``j+1``;
* a node with neither inputs nor outputs is skipped (isolated);
* a node without predecessors reads the stage input; otherwise the SUM of
  its predecessors' outputs; then Conv3x3('same') + ReLU;
* nodes without successors are summed into the DAG output;
* per stage: input conv (kernel_sizes[s]) + ReLU, then -- only if any bit
  is set -- the DAG and an output Conv3x3 + ReLU, then MaxPool 2x2/2;
* head: Flatten -> Dense(dense_units, ReLU) -> Dropout -> Dense(classes)
  -> softmax.

The decoded :class:`Plan` is a flat, topologically ordered list of conv
"layers" with explicit input-sum lists; both the torch oracle executor and
the HIP executor consume it, and it is cached by gene string (SURVEY.md §7.3
hard part 2).
"""

from collections import namedtuple

# A conv layer of the plan.
#   name     : unique id ("s1_in", "s1_n0", "s1_out", ...)
#   inputs   : list of tensor ids that are SUMMED to form the conv input
#   cin/cout : channels; k : (kh, kw) kernel size (odd, 'same' padding)
#   stage    : stage index
ConvSpec = namedtuple("ConvSpec", "name inputs cin cout k stage")
# A stage boundary: 2x2/2 max-pool of tensor ``src`` (sum of ``srcs``).
PoolSpec = namedtuple("PoolSpec", "name srcs stage")


def split_connections(bits):
    """'0101110011' -> ['0', '10', '111', '0011'] (chunk j has j+1 bits)."""
    chunks, i, n = [], 0, 1
    while i + n <= len(bits):
        chunks.append(bits[i:i + n])
        i += n
        n += 1
    if i != len(bits):
        raise ValueError("bit string of length {} is not K(K-1)/2".format(len(bits)))
    return chunks


def nodes_for_bits(nbits):
    k = 1
    while k * (k - 1) // 2 < nbits:
        k += 1
    if k * (k - 1) // 2 != nbits:
        raise ValueError("{} bits is not K(K-1)/2 for any K".format(nbits))
    return k


def decode_stage(bits, nodes):
    """Return ``(preds, succs, active, outputs)`` for one stage.

    ``preds[i]``: list of predecessor node ids of node i (empty = reads the
    stage input); ``active[i]``: node has inputs or outputs; ``outputs``:
    active nodes with no successors (summed into the DAG output).
    Raises IndexError for an all-zero string, like the reference's
    ``build_dag`` (the model builder skips the DAG in that case).
    """
    chunks = split_connections(bits)
    if len(chunks) != nodes - 1:
        raise ValueError("stage with {} nodes needs {} bits, got {}".format(
            nodes, nodes * (nodes - 1) // 2, len(bits)))
    preds = [[] for _ in range(nodes)]
    succs = [[] for _ in range(nodes)]
    for j, chunk in enumerate(chunks):        # chunk j -> inputs of node j+1
        for i, b in enumerate(chunk):
            if b == '1':
                preds[j + 1].append(i)
                succs[i].append(j + 1)
    active = [bool(preds[i] or succs[i]) for i in range(nodes)]
    outputs = [i for i in range(nodes) if active[i] and not succs[i]]
    if not outputs:
        raise IndexError("all-zero stage has no DAG (reference build_dag raises IndexError)")
    return preds, succs, active, outputs


class Plan(object):
    """Decoded Genetic-CNN architecture (topologically ordered)."""

    def __init__(self, genes, nodes, input_shape, kernels_per_layer, kernel_sizes, dense_units, classes):
        self.genes = dict(genes)
        self.nodes = tuple(nodes)
        self.input_shape = tuple(input_shape)        # (H, W, C) like Keras channels_last
        self.kernels_per_layer = tuple(kernels_per_layer)
        self.kernel_sizes = tuple(tuple(k) for k in kernel_sizes)
        self.dense_units = dense_units
        self.classes = classes
        self.steps = []          # ConvSpec / PoolSpec in execution order
        self._build()

    def _build(self):
        h, w, c = self.input_shape
        cur = "input"
        for s, cout in enumerate(self.kernels_per_layer):
            bits = self.genes["S_{}".format(s + 1)]
            k = self.kernel_sizes[s]
            if k[0] % 2 == 0 or k[1] % 2 == 0:
                raise ValueError("only odd kernel sizes are supported ('same' padding)")
            name_in = "s{}_in".format(s + 1)
            self.steps.append(ConvSpec(name_in, [cur], c, cout, tuple(k), s))
            cur = name_in
            if any(b == '1' for b in bits):
                preds, _succs, active, outputs = decode_stage(bits, self.nodes[s])
                for i in range(self.nodes[s]):
                    if not active[i]:
                        continue
                    srcs = [name_in] if not preds[i] else ["s{}_n{}".format(s + 1, p) for p in preds[i]]
                    self.steps.append(ConvSpec("s{}_n{}".format(s + 1, i), srcs, cout, cout, (3, 3), s))
                out_srcs = ["s{}_n{}".format(s + 1, i) for i in outputs]
                name_out = "s{}_out".format(s + 1)
                self.steps.append(ConvSpec(name_out, out_srcs, cout, cout, (3, 3), s))
                cur = name_out
            self.steps.append(PoolSpec("s{}_pool".format(s + 1), [cur], s))
            cur = "s{}_pool".format(s + 1)
            h, w, c = h // 2, w // 2, cout
        self.final_hw = (h, w)
        self.final_c = c
        self.flatten = h * w * c
        if self.flatten <= 0:
            raise ValueError("input too small for {} pooling stages".format(len(self.kernels_per_layer)))

    # ------------------------------------------------------------ accessors
    def convs(self):
        return [st for st in self.steps if isinstance(st, ConvSpec)]

    def stage_hw(self, stage):
        h, w, _ = self.input_shape
        return h >> stage, w >> stage

    def key(self):
        return (tuple(sorted(self.genes.items())), self.nodes, self.input_shape, self.kernels_per_layer,
                self.kernel_sizes, self.dense_units, self.classes)

    def describe(self):
        """Human-readable topology, e.g. for ``GeneticCnnModel.plot``."""
        lines = []
        for st in self.steps:
            if isinstance(st, ConvSpec):
                lines.append("{:8s} = relu(conv{}x{}({}->{})({}))".format(
                    st.name, st.k[0], st.k[1], st.cin, st.cout, " + ".join(st.inputs)))
            else:
                lines.append("{:8s} = maxpool2x2({})".format(st.name, " + ".join(st.srcs)))
        lines.append("dense1   = relu(dense({}->{}))".format(self.flatten, self.dense_units))
        lines.append("logits   = dense({}->{}) -> softmax".format(self.dense_units, self.classes))
        return "\n".join(lines)

    # ----------------------------------------------------------- cost model
    def forward_flops(self):
        """Forward FLOPs per sample (2*MAC), used by the LPT scheduler and the
        bench's FLOP accounting."""
        total = 0
        for st in self.convs():
            h, w = self.stage_hw(st.stage)
            total += 2 * h * w * st.cout * st.cin * st.k[0] * st.k[1]
        total += 2 * self.flatten * self.dense_units + 2 * self.dense_units * self.classes
        return total

    def param_count(self):
        n = sum(st.cout * st.cin * st.k[0] * st.k[1] + st.cout for st in self.convs())
        n += self.flatten * self.dense_units + self.dense_units
        n += self.dense_units * self.classes + self.classes
        return n


_PLAN_CACHE = {}


def make_plan(genes, nodes, input_shape, kernels_per_layer, kernel_sizes, dense_units, classes):
    key = (tuple(sorted(genes.items())), tuple(nodes), tuple(input_shape), tuple(kernels_per_layer),
           tuple(tuple(k) for k in kernel_sizes), dense_units, classes)
    plan = _PLAN_CACHE.get(key)
    if plan is None:
        plan = Plan(genes, nodes, input_shape, kernels_per_layer, kernel_sizes, dense_units, classes)
        if len(_PLAN_CACHE) > 4096:
            _PLAN_CACHE.clear()
        _PLAN_CACHE[key] = plan
    return plan

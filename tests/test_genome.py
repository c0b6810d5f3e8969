"""Genetic-CNN decoding test vectors (reference
gentun/models/keras_models.py:46-118)."""

import pytest

from gentun_amd import GeneticCnnModel
from gentun_amd.models.genome import ConvSpec, decode_stage, make_plan, split_connections


def dag(bits, nodes):
    """-> {node: sorted predecessor list ('X' = stage input)}, outputs."""
    preds, _succs, active, outputs = decode_stage(bits, nodes)
    return {i: (preds[i] or ['X']) for i in range(nodes) if active[i]}, outputs


def test_split_connections():
    assert split_connections('0101110011') == ['0', '10', '111', '0011']
    with pytest.raises(ValueError):
        split_connections('01')


@pytest.mark.parametrize("bits,nodes,expect,outs", [
    ('1', 2, {0: ['X'], 1: [0]}, [1]),
    ('101', 3, {0: ['X'], 1: [0], 2: [1]}, [2]),
    ('100', 3, {0: ['X'], 1: [0]}, [1]),
    ('010', 3, {0: ['X'], 2: [0]}, [2]),
    ('001', 3, {1: ['X'], 2: [1]}, [2]),
    ('111', 3, {0: ['X'], 1: [0], 2: [0, 1]}, [2]),
    ('110', 3, {0: ['X'], 1: [0], 2: [0]}, [1, 2]),
    ('1000000000', 5, {0: ['X'], 1: [0]}, [1]),
    ('0101110011', 5, {0: ['X'], 1: ['X'], 2: [0], 3: [0, 1, 2], 4: [2, 3]}, [4]),
    ('1111111111', 5, {0: ['X'], 1: [0], 2: [0, 1], 3: [0, 1, 2], 4: [0, 1, 2, 3]}, [4]),
    # traced by hand through keras_models.py:51-74 (chunks '1','00','100','1001'):
    # node 2 is isolated and node 4 = C(n0 + n3). SURVEY App. A.1 lists a
    # different DAG for this string; the reference code gives this one.
    ('1001001001', 5, {0: ['X'], 1: [0], 3: [0], 4: [0, 3]}, [1, 4]),
])
def test_decode_vectors(bits, nodes, expect, outs):
    got, outputs = dag(bits, nodes)
    assert got == expect
    assert outputs == outs


def test_all_zero_stage():
    with pytest.raises(IndexError):
        decode_stage('000', 3)
    plan = make_plan({'S_1': '000', 'S_2': '0000000000'}, (3, 5), (28, 28, 1), (20, 50), ((5, 5), (5, 5)), 500, 10)
    names = [st.name for st in plan.steps]
    assert names == ['s1_in', 's1_pool', 's2_in', 's2_pool']


def test_plan_topology_and_output_conv():
    plan = make_plan({'S_1': '110', 'S_2': '0101110011'}, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
    convs = {st.name: st for st in plan.steps if isinstance(st, ConvSpec)}
    assert convs['s1_out'].inputs == ['s1_n1', 's1_n2']         # DAG outputs summed into the output conv
    assert convs['s2_n3'].inputs == ['s2_n0', 's2_n1', 's2_n2']
    assert convs['s2_in'].k == (5, 5) and convs['s2_n0'].k == (3, 3)
    assert plan.flatten == 8 * 8 * 50


@pytest.mark.parametrize("genes,shape,kernels,ks,mflop,params", [
    ({'S_1': '000', 'S_2': '0000000000'}, (28, 28, 1), (20, 50), ((5, 5), (5, 5)), 13.04, 1.256e6),
    ({'S_1': '111', 'S_2': '1111111111'}, (28, 28, 1), (20, 50), ((5, 5), (5, 5)), 88.54, 1.406e6),
    ({'S_1': '111', 'S_2': '1111111111'}, (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 117.69, 1.782e6),
])
def test_cost_model_matches_appendix(genes, shape, kernels, ks, mflop, params):
    plan = make_plan(genes, (3, 5), shape, kernels, ks, 500, 10)
    assert abs(plan.forward_flops() / 1e6 - mflop) < 0.01
    assert abs(plan.param_count() - params) / params < 1e-3


def test_deep_config_cost():
    genes = {'S_1': '111', 'S_2': '111111', 'S_3': '1111111111'}
    plan = make_plan(genes, (3, 4, 5), (32, 32, 3), (64, 128, 256), ((3, 3),) * 3, 500, 10)
    assert abs(plan.forward_flops() / 1e6 - 1215.6) < 1.0
    assert abs(plan.param_count() - 6.850e6) / 6.85e6 < 1e-3


def test_model_api_build_dag_and_plot(tmp_path):
    body, out = GeneticCnnModel.build_dag('X', 5, '0101110011', 50)
    assert [n for n, _ in body] == ['n0', 'n1', 'n2', 'n3', 'n4'] and out == 'n4'
    assert body[3][1] == 'relu(conv3x3x50(n0 + n1 + n2))'
    with pytest.raises(IndexError):
        GeneticCnnModel.build_dag('X', 3, '000', 20)
    m = GeneticCnnModel(None, None, {'S_1': '101', 'S_2': '0000000001'}, (3, 5), (28, 28, 1), (20, 50),
                        ((5, 5), (5, 5)), 500, 0.5, 10, device='cpu')
    p = m.plot(str(tmp_path / "net.txt"))
    assert "maxpool2x2" in open(p).read()
    assert m.name == '101-0000000001'


def test_epochs_learning_rate_rules():
    args = (None, None, {'S_1': '101', 'S_2': '0000000001'}, (3, 5), (28, 28, 1), (20, 50), ((5, 5), (5, 5)),
            500, 0.5, 10)
    GeneticCnnModel(*args, epochs=(2, 1), learning_rate=(1e-3, 1e-4), device='cpu')
    GeneticCnnModel(*args, epochs=3, learning_rate=1e-3, device='cpu')      # Q7: int epochs + float lr ok
    with pytest.raises(ValueError):
        GeneticCnnModel(*args, epochs=[2], learning_rate=[1e-3], device='cpu')
    with pytest.raises(ValueError):
        GeneticCnnModel(*args, epochs=(2,), learning_rate=1e-3, device='cpu')
    with pytest.raises(ValueError):
        GeneticCnnModel(*args, epochs=(2, 1), learning_rate=(1e-3,), device='cpu')


def test_plot_writes_graph_images(tmp_path):
    """plot(): the reference writes <name>.png (keras_models.py:41-44); PNG, SVG and DOT here."""
    import zlib
    m = GeneticCnnModel(None, None, {'S_1': '111', 'S_2': '0101110011'}, (3, 5), (32, 32, 3), (20, 50),
                        ((5, 5), (5, 5)), 500, 0.5, 10, device='cpu')
    png = open(m.plot(str(tmp_path / "net.png")), "rb").read()
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    import struct
    w, h = struct.unpack(">II", png[16:24])
    idat = png[png.index(b"IDAT") + 4:png.index(b"IEND") - 8]
    raw = zlib.decompress(idat)
    assert len(raw) == h * (w + 1) and w > 100 and h > 100
    assert 0 in raw[1:] and 255 in raw                                  # ink on a white canvas
    svg = open(m.plot(str(tmp_path / "net.svg"))).read()
    # s2 node 3 sums n0 + n1 + n2 through an add node; 12 convs + 2 pools + head
    assert "s2_n3_add" not in svg and svg.count("<rect") == 1 + svg.count("<text")
    dot = open(m.plot(str(tmp_path / "net.dot"))).read()
    for e in ('"s2_n0" -> "s2_n3_add"', '"s2_n1" -> "s2_n3_add"', '"s2_n2" -> "s2_n3_add"', '"s2_n3_add" -> "s2_n3"',
              '"s1_out" -> "s1_pool"', '"dense1" -> "dropout"'):
        assert e in dot, e


def test_reset_weights_redraws_kernels_keeps_biases():
    """reset_weights (keras_models.py:120-125): kernels re-drawn, biases kept."""
    import torch
    from gentun_amd.utils.data import make_cifar_like
    x, y = make_cifar_like(n=48, seed=1)
    m = GeneticCnnModel(x, y, {'S_1': '1', 'S_2': '1'}, (2, 2), x.shape[1:], (4, 4), ((3, 3), (3, 3)), 8, 0.5, 10,
                        nfold=2, epochs=(1,), learning_rate=(1e-2,), batch_size=16, backend="torch",
                        device=torch.device("cpu"), reset="all")
    assert m.reset_weights() == 0                     # nothing trained yet
    m.cross_validate()
    job = m.jobs[0]
    views = job._views()
    before = {k: v.clone() for k, v in views.items()}
    assert m.reset_weights() == 1
    after = job._views()
    kinds = {name: kind for name, _, kind, _ in job.shapes}
    for name, kind in kinds.items():
        if kind == "glorot":
            assert not torch.equal(before[name], after[name]), name
        else:
            assert torch.equal(before[name], after[name]), name
    assert any(before[n].abs().sum() > 0 for n, k in kinds.items() if k == "zero")    # trained biases kept


def test_reset_weights_counts_shared_fold_models_once():
    """Sequential folds (reset='kernels'): the per-fold jobs of one SequentialFoldJob may share one set of
    buffers (fold reuse); reset_weights re-draws each distinct model once and reports how many it reset."""
    import torch
    from gentun_amd.utils.data import make_cifar_like
    x, y = make_cifar_like(n=48, seed=1)
    m = GeneticCnnModel(x, y, {'S_1': '1', 'S_2': '1'}, (2, 2), x.shape[1:], (4, 4), ((3, 3), (3, 3)), 8, 0.5, 10,
                        nfold=2, epochs=(1,), learning_rate=(1e-2,), batch_size=16, backend="torch",
                        device=torch.device("cpu"), reset="kernels")
    m.cross_validate()
    folds = [j for job in m.jobs for j in (getattr(job, "jobs", None) or [job])]
    distinct = {j.flat.data_ptr() for j in folds}
    assert m.reset_weights() == len(distinct) == len(m._live_jobs())

"""``GeneticCnnModel`` -- reference-compatible fitness model for Genetic-CNN.

API parity with gentun/models/keras_models.py:19-143 (constructor signature,
``build_model``, static ``build_dag``, ``reset_weights``, ``plot``,
``cross_validate``); the Keras/TF graph is replaced by a decoded
:class:`~gentun_amd.models.genome.Plan` executed by the fold-batched engine
(:mod:`gentun_amd.models.cnn_engine`) -- HIP kernels on MI355X.
"""

import torch

from ..utils.data import labels_from_onehot, stratified_kfold
from .generic_models import GentunModel
from .genome import decode_stage, make_plan
from . import cnn_engine as _eng


def _pick_device(device):
    if device is not None:
        return torch.device(device)
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class GeneticCnnModel(GentunModel):

    def __init__(self, x_train, y_train, genes, nodes, input_shape, kernels_per_layer, kernel_sizes, dense_units,
                 dropout_probability, classes, nfold=5, epochs=(3,), learning_rate=(1e-3,), batch_size=32,
                 loss="bce_compat", dtype="fp32", seed=0, backend=None, device=None, fold_parallel=True,
                 optimizer="adam", momentum=0.9, reset="kernels", batching="keras", batch_norm=False,
                 verbose=False, pad_images=True):
        super(GeneticCnnModel, self).__init__(x_train, y_train)
        self.genes = dict(genes)
        self.name = '-'.join(self.genes[k] for k in sorted(self.genes))
        # Reference type rules (keras_models.py:30-38), relaxed per SURVEY.md Q7:
        # int epochs may come with an int OR float learning rate.
        if isinstance(epochs, (list, tuple)) != isinstance(learning_rate, (list, tuple)):
            raise ValueError("epochs and learning_rate must both be scalars or both be tuples")
        if isinstance(epochs, list) or isinstance(learning_rate, list):
            raise ValueError("epochs and learning_rate must be tuples (lists are rejected like the reference)")
        if not isinstance(epochs, tuple):
            epochs, learning_rate = (int(epochs),), (float(learning_rate),)
        if len(epochs) != len(learning_rate):
            raise ValueError("epochs and learning_rate tuples must have the same length")
        self.nodes = tuple(nodes)
        self.input_shape = tuple(input_shape)
        self.kernels_per_layer = tuple(kernels_per_layer)
        self.kernel_sizes = tuple(tuple(k) for k in kernel_sizes)
        self.dense_units = dense_units
        self.dropout_probability = dropout_probability
        self.classes = classes
        self.nfold = nfold
        self.epochs = epochs
        self.learning_rate = learning_rate
        self.batch_size = batch_size
        self.device = _pick_device(device)
        self.backend = backend or _eng.default_backend(self.device)
        self.cfg = _eng.TrainConfig(epochs=epochs, learning_rate=learning_rate, batch_size=batch_size,
                                    dropout=dropout_probability, loss=loss, dtype=dtype, seed=seed,
                                    optimizer=optimizer, momentum=momentum, reset=reset, batching=batching,
                                    batch_norm=batch_norm, verbose=verbose, nfold=nfold, pad_images=pad_images)
        self.fold_parallel = fold_parallel
        self.model = self.build_model(self.genes, self.nodes, self.input_shape, self.kernels_per_layer,
                                      self.kernel_sizes, self.dense_units, self.dropout_probability, self.classes)
        self.fold_scores = []
        self.fold_metrics = None
        self.jobs = []               # the trained job(s) of the last cross_validate (reset_weights)

    # ------------------------------------------------------------ structure
    def build_model(self, genes, nodes, input_shape, kernels_per_layer, kernel_sizes, dense_units,
                    dropout_probability, classes):
        """Decode genes into an executable plan (keras_models.py:97-118)."""
        return make_plan(genes, nodes, input_shape, kernels_per_layer, kernel_sizes, dense_units, classes)

    @staticmethod
    def build_dag(x, nodes, connections, kernels):
        """Symbolic DAG of one stage (keras_models.py:46-95): returns the
        list of ``(node, input_expr)`` and the output expression, with
        ``x`` as the stage-input name. Raises IndexError on all-zero bits."""
        preds, _succs, active, outputs = decode_stage(connections, nodes)
        names = {}
        body = []
        for i in range(nodes):
            if not active[i]:
                continue
            src = x if not preds[i] else " + ".join(names[p] for p in preds[i])
            names[i] = "n{}".format(i)
            body.append((names[i], "relu(conv3x3x{}({}))".format(kernels, src)))
        return body, " + ".join(names[i] for i in outputs)

    def reset_weights(self):
        """keras_models.py:120-125: re-run the kernel initialisers of the
        model's live weights, keeping the biases (and BatchNorm state). The
        weights live in the job(s) the last :meth:`cross_validate` trained
        (one per fold with the reference's sequential folds); before any
        training there is nothing to reset -- every job draws fresh Glorot
        kernels when it starts, which is the same policy. Returns the number
        of jobs whose kernels were re-drawn."""
        n = 0
        for job in self._live_jobs():
            job.reset_kernels()
            n += 1
        return n

    def _live_jobs(self):
        """The distinct models behind the last training: a SequentialFoldJob holds one job per fold, but
        with fold reuse (the HIP default) those are shallow copies sharing ONE set of device buffers --
        counted once (the last fold's job: its seeds are the ones the buffers were last re-pointed to)."""
        seen = {}
        for job in self.jobs:
            for j in (getattr(job, "jobs", None) or [job]):     # SequentialFoldJob: one job per fold
                flat = getattr(j, "flat", None)
                seen[flat.data_ptr() if flat is not None else id(j)] = j
        return list(seen.values())

    def plot(self, path=None):
        """Draw the decoded network to validate gene-to-DAG (keras_models.py:
        41-44 writes ``<name>.png`` with Keras' plot_model). ``path`` suffix
        ``.png`` (default), ``.svg`` or ``.dot``; ``.txt`` writes the textual
        topology. Returns the path."""
        from ..utils.plot import plot_plan
        path = path or "{}.png".format(self.name)
        if path.lower().endswith(".txt"):
            with open(path, "w") as f:
                f.write(self.model.describe() + "\n")
            return path
        return plot_plan(self.model, path)

    # ------------------------------------------------------------ training
    def make_folds(self):
        labels = labels_from_onehot(self.y_train)
        return stratified_kfold(labels, self.nfold, seed=self.cfg.seed)

    def member(self, fold_ids=None):
        """``(plan, folds, fold_ids)`` of this candidate for a population job."""
        folds = self.make_folds()
        ids = list(range(self.nfold)) if fold_ids is None else list(fold_ids)
        return (self.model, [folds[i] for i in ids], ids)

    def make_jobs(self, stream=None, fold_ids=None):
        folds = self.make_folds()
        ids = list(range(self.nfold)) if fold_ids is None else list(fold_ids)
        # sequential-fold semantics need every fold of the candidate in one job
        groups = [ids] if (self.fold_parallel or self.cfg.reset == "kernels") else [[i] for i in ids]
        return [_eng.make_job(self.backend, self.model, self.x_train, self.y_train, [folds[i] for i in grp],
                              self.cfg, self.device, fold_ids=grp, stream=stream) for grp in groups]

    def primary_metric(self):
        return "binary_accuracy" if self.cfg.loss == "bce_compat" else "categorical_accuracy"

    def collect(self, results):
        """Merge per-job results (in fold order) into fitness."""
        merged = {"val_loss": [], "binary_accuracy": [], "categorical_accuracy": []}
        for res in results:
            for k in merged:
                merged[k].extend(res[k])
        self.fold_metrics = merged
        self.fold_scores = list(merged[self.primary_metric()])
        return sum(self.fold_scores) / len(self.fold_scores)

    def cross_validate(self):
        """Mean validation metric over ``nfold`` folds (keras_models.py:127-143)."""
        jobs = self.make_jobs()
        results = []
        for job in jobs:
            job.launch()
            results.append(job.finish())
        self.jobs = jobs
        return self.collect(results)

"""Individuals: genome encoding, GA operators and lazily-evaluated fitness.

Behavioural parity targets (reference = jedison-github/gentun @ v0):

* ``random_log_uniform``            -- gentun/individuals.py:23-35
* ``Individual`` base + operators   -- gentun/individuals.py:38-153
* ``XgboostIndividual``             -- gentun/individuals.py:156-216
* ``GeneticCnnIndividual``          -- gentun/individuals.py:219-284

All randomness goes through :mod:`gentun_amd.utils.rng` (a process-wide
``random.Random`` that defaults to an OS-seeded state, exactly like the
reference's use of the global ``random`` module, but which can be seeded and
checkpointed -- SURVEY.md Q12).

Fitness evaluation itself is delegated to the model layer
(:mod:`gentun_amd.models`), which runs on MI355X (HIP kernels) for the
Genetic-CNN species and on the native C++/HIP GBDT engine for the XGBoost
species.
"""

import math
import pprint

from .utils import rng as _rng


def random_log_uniform(minimum, maximum, base, eps=1e-12):
    """Sample ``[minimum, maximum]`` uniformly on a log scale.

    ``base == 0``  -> plain uniform sample.
    ``base > 0``   -> log-uniform between ``minimum + eps`` and ``maximum``.
    ``base < 0``   -> "reverse" log scale: ``maximum - |base|**U`` so that the
                      mass concentrates next to ``maximum`` (used for the
                      subsample / colsample genes).
    (reference: gentun/individuals.py:23-35)
    """
    r = _rng.get()
    if base == 0:
        return r.uniform(minimum, maximum)
    lo = minimum + eps
    if base > 0:
        exponent = r.uniform(math.log(lo, base), math.log(maximum, base))
        return base ** exponent
    b = -base
    exponent = r.uniform(math.log(eps, b), math.log(maximum - lo, b))
    return maximum - b ** exponent


def _sample_gene(spec):
    """Draw one gene value from an XGBoost-style ``(default, min, max, base)`` spec."""
    default, minimum, maximum, base = spec
    if isinstance(default, int) and not isinstance(default, bool):
        return _rng.get().randint(minimum, maximum)
    return round(random_log_uniform(minimum, maximum, base), 4)


class Individual(object):
    """Genome container with GA operators and memoised fitness.

    Subclasses define ``generate_random_genes``, ``evaluate_fitness`` and
    ``get_additional_parameters`` (reference: gentun/individuals.py:38-153).
    """

    def __init__(self, x_train, y_train, genome, genes, crossover_rate, mutation_rate,
                 additional_parameters=None):
        self.x_train = x_train
        self.y_train = y_train
        self.genome = genome
        self.validate_genome()
        self.genes = genes
        self.validate_genes()
        self.crossover_rate = crossover_rate
        self.mutation_rate = mutation_rate
        self.fitness = None
        # Optional per-fold detail filled by evaluators (not part of the ref API).
        self.fold_scores = None
        if additional_parameters is not None:
            raise AssertionError("additional_parameters must be passed as subclass keyword arguments")

    # ------------------------------------------------------------------ checks
    def validate_genome(self):
        if not isinstance(self.genome, dict):
            raise TypeError("Genome must be a dictionary.")
        for name in self.genome:
            if not isinstance(name, str):
                raise TypeError("Gene names must be strings.")

    def validate_genes(self):
        if set(self.genes) != set(self.genome):
            raise ValueError("Genes passed don't correspond to individual's genome.")

    # ----------------------------------------------------------------- getters
    def get_genes(self):
        return self.genes

    def get_genome(self):
        return self.genome

    @staticmethod
    def generate_random_genes(genome):
        raise NotImplementedError("Use a subclass with genes definition.")

    def evaluate_fitness(self):
        raise NotImplementedError("Use a subclass with genes definition.")

    def get_additional_parameters(self):
        raise NotImplementedError("Use a subclass with genes definition.")

    def get_fitness(self):
        """Evaluate on first access, then return the memoised value."""
        if self.fitness is None:
            self.evaluate_fitness()
        return self.fitness

    def get_fitness_status(self):
        return self.fitness is not None

    def set_fitness(self, value):
        self.fitness = value
        if value is None:
            self.fold_scores = None
            self.fold_metrics = None

    # --------------------------------------------------------------- operators
    def _spawn(self, genes):
        return self.__class__(self.x_train, self.y_train, self.genome, genes,
                              self.crossover_rate, self.mutation_rate,
                              **self.get_additional_parameters())

    def reproduce(self, partner):
        """Uniform crossover into a NEW child (parents untouched).

        Each gene comes from ``partner`` with probability ``crossover_rate``.
        (reference: gentun/individuals.py:94-109)
        """
        if self.__class__ is not partner.__class__:
            raise AssertionError("Individuals of different species cannot reproduce")
        r = _rng.get()
        mine, theirs = self.get_genes(), partner.get_genes()
        child = {}
        for name, value in mine.items():
            child[name] = theirs[name] if r.random() < self.crossover_rate else value
        return self._spawn(child)

    def crossover(self, partner):
        """In-place uniform gene swap between ``self`` and ``partner``.
        (reference: gentun/individuals.py:111-121)
        """
        if self.__class__ is not partner.__class__:
            raise AssertionError("Individuals of different species cannot cross")
        r = _rng.get()
        mine, theirs = self.get_genes(), partner.get_genes()
        for name in list(mine):
            if r.random() < self.crossover_rate:
                mine[name], theirs[name] = theirs[name], mine[name]
                self.set_fitness(None)
                partner.set_fitness(None)

    def mutate(self):
        """Re-sample each gene from its prior with probability ``mutation_rate``.
        (reference: gentun/individuals.py:123-132)
        """
        r = _rng.get()
        genes = self.get_genes()
        for name in list(genes):
            if r.random() < self.mutation_rate:
                genes[name] = _sample_gene(self.get_genome()[name])
                self.set_fitness(None)

    def copy(self):
        """Copy genes (shallow dict copy) and keep the memoised fitness."""
        twin = self._spawn(dict(self.genes))
        twin.set_fitness(self.fitness)
        twin.fold_scores = None if self.fold_scores is None else list(self.fold_scores)
        fm = getattr(self, "fold_metrics", None)
        if fm:
            twin.fold_metrics = {k: list(v) for k, v in fm.items()}
        return twin

    def genes_key(self):
        """Hashable identity of the genes (used by optional fitness caches)."""
        return tuple(sorted((k, str(v)) for k, v in self.genes.items()))

    def __str__(self):
        return pprint.pformat(self.genes)


# ---------------------------------------------------------------------------
# XGBoost-style GBDT hyper-parameter individual
# ---------------------------------------------------------------------------

def default_xgboost_genome():
    """Gene priors ``name: (default, min, max, log_base)``
    (reference: gentun/individuals.py:162-175)."""
    return {
        'eta': (0.3, 0.001, 1.0, 10),
        'min_child_weight': (1, 0, 10, None),
        'max_depth': (6, 3, 10, None),
        'gamma': (0.0, 0.0, 10.0, 10),
        'max_delta_step': (0, 0, 10, None),
        'subsample': (1.0, 0.0, 1.0, -10),
        'colsample_bytree': (1.0, 0.0, 1.0, -10),
        'colsample_bylevel': (1.0, 0.0, 1.0, -10),
        'lambda': (1.0, 0.1, 10.0, 10),
        'alpha': (0.0, 0.0, 10.0, 10),
        'scale_pos_weight': (1.0, 0.0, 10.0, 0),
    }


class XgboostIndividual(Individual):
    """GBDT hyper-parameter individual; fitness = k-fold CV metric of the
    native GBDT engine (reference: gentun/individuals.py:156-216)."""

    def __init__(self, x_train, y_train, genome=None, genes=None, crossover_rate=0.5, mutation_rate=0.015,
                 booster='gbtree', objective='reg:linear', eval_metric='rmse', nfold=5,
                 num_boost_round=5000, early_stopping_rounds=100, device=None, seed=0):
        if genome is None:
            genome = default_xgboost_genome()
        if genes is None:
            genes = self.generate_random_genes(genome)
        super(XgboostIndividual, self).__init__(x_train, y_train, genome, genes, crossover_rate, mutation_rate)
        self.booster = booster
        self.objective = objective
        self.eval_metric = eval_metric
        self.nfold = nfold
        self.num_boost_round = num_boost_round
        self.early_stopping_rounds = early_stopping_rounds
        self.device = device
        self.seed = seed

    @staticmethod
    def generate_random_genes(genome):
        return {name: _sample_gene(spec) for name, spec in genome.items()}

    def evaluate_fitness(self):
        from .models.xgboost_models import XgboostModel
        model = XgboostModel(self.x_train, self.y_train, self.genes, booster=self.booster,
                             objective=self.objective, eval_metric=self.eval_metric, nfold=self.nfold,
                             num_boost_round=self.num_boost_round,
                             early_stopping_rounds=self.early_stopping_rounds,
                             device=self.device, seed=self.seed)
        self.fitness = model.cross_validate()

    def get_additional_parameters(self):
        return {
            'booster': self.booster,
            'objective': self.objective,
            'eval_metric': self.eval_metric,
            'nfold': self.nfold,
            'num_boost_round': self.num_boost_round,
            'early_stopping_rounds': self.early_stopping_rounds,
            'device': self.device,
            'seed': self.seed,
        }


# ---------------------------------------------------------------------------
# Genetic-CNN architecture individual
# ---------------------------------------------------------------------------

class GeneticCnnIndividual(Individual):
    """Genetic-CNN individual: one bit-string gene ``S_s`` of ``K_s(K_s-1)/2``
    bits per stage (reference: gentun/individuals.py:219-284).

    Extra keyword arguments beyond the reference signature (all optional):
    ``loss`` ('bce_compat' = Keras softmax+binary_crossentropy parity, or 'ce'),
    ``dtype`` ('fp32', the reference precision: fp32 tensors, exact split-fp32 MFMA on
    MI355X; or 'bf16', the fast mode: bf16 tensors and MFMA, fp32 master weights), ``seed``
    (run seed; fitness is a pure function of (genes, seed, fold)),
    ``backend`` ('hip' -- MI355X kernels, default on GPU -- or 'torch' oracle),
    ``device``, ``optimizer`` ('adam' = the reference's Keras Adam, or
    'sgd' = Keras SGD with ``momentum``; both reset at every lr stage),
    ``reset`` ('kernels' = the reference's sequential folds that re-draw only
    the kernels, or 'all' = concurrent folds from fresh weights) and
    ``batching`` ('keras' = short last batch, or 'wrap') and ``batch_norm``
    (False = the reference network; True = conv -> BatchNorm -> ReLU in every
    node, Keras BatchNormalization defaults) and ``verbose`` (print the
    reference's "KFold i/n" / "Training N epochs with learning rate lr" lines,
    keras_models.py:134,137).
    """

    def __init__(self, x_train, y_train, genome=None, genes=None, crossover_rate=0.3, mutation_rate=0.1,
                 nodes=(3, 5), input_shape=(28, 28, 1), kernels_per_layer=(20, 50),
                 kernel_sizes=((5, 5), (5, 5)), dense_units=500, dropout_probability=0.5, classes=10,
                 nfold=5, epochs=(3,), learning_rate=(1e-3,), batch_size=32,
                 loss='bce_compat', dtype='fp32', seed=0, backend=None, device=None, optimizer='adam',
                 momentum=0.9, reset='kernels', batching='keras', batch_norm=False, verbose=False,
                 pad_images=True):
        if genome is None:
            genome = {'S_{}'.format(i + 1): k * (k - 1) // 2 for i, k in enumerate(nodes)}
        if genes is None:
            genes = self.generate_random_genes(genome)
        super(GeneticCnnIndividual, self).__init__(x_train, y_train, genome, genes, crossover_rate, mutation_rate)
        if not (len(nodes) == len(kernels_per_layer) == len(kernel_sizes)):
            raise AssertionError("nodes, kernels_per_layer and kernel_sizes must have equal length")
        for name, bits in self.genes.items():
            if len(bits) != self.genome[name]:
                raise AssertionError("gene {} has {} bits, genome expects {}".format(name, len(bits), self.genome[name]))
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
        self.loss = loss
        self.dtype = dtype
        self.seed = seed
        self.backend = backend
        self.device = device
        self.optimizer = optimizer
        self.momentum = momentum
        self.reset = reset
        self.batching = batching
        self.batch_norm = batch_norm
        self.verbose = verbose
        # HIP executor: 28 x 28 stored zero-padded to 32 x 32 for the shape-specialised kernels
        self.pad_images = bool(pad_images)

    @staticmethod
    def generate_random_genes(genome):
        r = _rng.get()
        return {name: ''.join('1' if r.random() < 0.5 else '0' for _ in range(nbits))
                for name, nbits in genome.items()}

    def build_fitness_model(self, device=None):
        """The fitness model for these genes (lets batch evaluators enqueue
        several candidates on different HIP streams)."""
        from .models.cnn import GeneticCnnModel
        return GeneticCnnModel(self.x_train, self.y_train, self.genes, self.nodes, self.input_shape,
                               self.kernels_per_layer, self.kernel_sizes, self.dense_units,
                               self.dropout_probability, self.classes, self.nfold, self.epochs,
                               self.learning_rate, self.batch_size, loss=self.loss, dtype=self.dtype,
                               seed=self.seed, backend=self.backend, device=device or self.device,
                               optimizer=self.optimizer, momentum=self.momentum, reset=self.reset,
                               batching=self.batching, batch_norm=self.batch_norm,
                               verbose=self.verbose, pad_images=self.pad_images)

    def cost(self):
        """Relative training cost (forward FLOPs/sample); LPT scheduling key."""
        from .models.genome import make_plan
        return make_plan(self.genes, self.nodes, self.input_shape, self.kernels_per_layer, self.kernel_sizes,
                         self.dense_units, self.classes).forward_flops()

    def evaluate_fitness(self):
        model = self.build_fitness_model()
        self.fitness = model.cross_validate()
        self.fold_scores = list(model.fold_scores)
        self.fold_metrics = dict(model.fold_metrics or {})

    def get_additional_parameters(self):
        return {
            'nodes': self.nodes,
            'input_shape': self.input_shape,
            'kernels_per_layer': self.kernels_per_layer,
            'kernel_sizes': self.kernel_sizes,
            'dense_units': self.dense_units,
            'dropout_probability': self.dropout_probability,
            'classes': self.classes,
            'nfold': self.nfold,
            'epochs': self.epochs,
            'learning_rate': self.learning_rate,
            'batch_size': self.batch_size,
            'loss': self.loss,
            'dtype': self.dtype,
            'seed': self.seed,
            'backend': self.backend,
            'device': self.device,
            'optimizer': self.optimizer,
            'momentum': self.momentum,
            'reset': self.reset,
            'batching': self.batching,
            'batch_norm': self.batch_norm,
            'verbose': self.verbose,
            'pad_images': self.pad_images,
        }

    def mutate(self):
        """Flip every bit independently with probability ``mutation_rate``;
        fitness resets only if a string actually changed
        (reference: gentun/individuals.py:276-284)."""
        r = _rng.get()
        genes = self.get_genes()
        for name in list(genes):
            old = genes[name]
            new = ''.join(('1' if c == '0' else '0') if r.random() < self.mutation_rate else c for c in old)
            if new != old:
                self.set_fitness(None)
                genes[name] = new

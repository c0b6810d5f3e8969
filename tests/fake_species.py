"""Analytic test species: instant, deterministic fitness so GA / distribution
logic can be tested in milliseconds (SURVEY.md §4 recommendation 2)."""

from gentun_amd.individuals import Individual, _sample_gene
from gentun_amd.utils import rng as _rng

EVALS = {"n": 0}


class BitIndividual(Individual):
    """Genome: bit-string genes; fitness = popcount (maximise)."""

    def __init__(self, x_train, y_train, genome=None, genes=None, crossover_rate=0.5, mutation_rate=0.1,
                 nfold=1):
        if genome is None:
            genome = {'A': 6, 'B': 4}
        if genes is None:
            genes = self.generate_random_genes(genome)
        super(BitIndividual, self).__init__(x_train, y_train, genome, genes, crossover_rate, mutation_rate)
        self.nfold = nfold

    @staticmethod
    def generate_random_genes(genome):
        r = _rng.get()
        return {k: ''.join('1' if r.random() < 0.5 else '0' for _ in range(n)) for k, n in genome.items()}

    def evaluate_fitness(self):
        EVALS["n"] += 1
        self.fitness = float(sum(v.count('1') for v in self.genes.values()))
        self.fold_scores = [self.fitness]

    def get_additional_parameters(self):
        return {'nfold': self.nfold}

    def mutate(self):
        r = _rng.get()
        for name in list(self.genes):
            old = self.genes[name]
            new = ''.join(('1' if c == '0' else '0') if r.random() < self.mutation_rate else c for c in old)
            if new != old:
                self.genes[name] = new
                self.set_fitness(None)

    def cost(self):
        return 1.0 + sum(v.count('1') for v in self.genes.values())


class NumIndividual(Individual):
    """Tuple-spec genome; fitness = (x - 3)^2 + (y - 0.25)^2 (minimise)."""

    def __init__(self, x_train, y_train, genome=None, genes=None, crossover_rate=0.5, mutation_rate=0.2):
        if genome is None:
            genome = {'x': (1, 0, 10, None), 'y': (0.5, 0.0, 1.0, 0)}
        if genes is None:
            genes = {k: _sample_gene(v) for k, v in genome.items()}
        super(NumIndividual, self).__init__(x_train, y_train, genome, genes, crossover_rate, mutation_rate)

    @staticmethod
    def generate_random_genes(genome):
        return {k: _sample_gene(v) for k, v in genome.items()}

    def evaluate_fitness(self):
        EVALS["n"] += 1
        self.fitness = (self.genes['x'] - 3) ** 2 + (self.genes['y'] - 0.25) ** 2

    def get_additional_parameters(self):
        return {}


class FlakyBitIndividual(BitIndividual):
    """A BitIndividual whose evaluation ALWAYS raises when gene 'A' starts
    with '11' (so the rank-0 re-evaluation fails too)."""

    FAILS = [0]

    def evaluate_fitness(self):
        if self.genes['A'].startswith('11'):
            FlakyBitIndividual.FAILS[0] += 1
            raise RuntimeError("permanent evaluation failure")
        super(FlakyBitIndividual, self).evaluate_fitness()


class SlowBitIndividual(BitIndividual):
    """A BitIndividual whose evaluation takes 20 ms: under the dynamic (work-stealing) schedule every
    rank then gets units to claim, however fast rank 0 leaves its broadcast."""

    def evaluate_fitness(self):
        import time
        time.sleep(0.02)
        super(SlowBitIndividual, self).evaluate_fitness()

"""Populations: containers of same-species individuals plus fittest selection.

Reference parity: gentun/populations.py:10-67 (``Population``) and :70-105
(``GridPopulation``).

MI355X-first extension: a population may carry an *evaluator* strategy
(:mod:`gentun_amd.parallel.evaluators`). When present, ``get_fittest`` first
hands every not-yet-evaluated individual to the evaluator in ONE batch (so a
GPU can train several candidates concurrently, or ranks can split them)
instead of the reference's strictly sequential lazy loop
(gentun/populations.py:55-58). Without an evaluator the behaviour is the
reference's. The evaluator travels with every population derived from this
one (``empty_like``), which fixes the reference bug where next generations
silently drop their distribution settings.
"""

import itertools
import operator


class Population(object):

    def __init__(self, species, x_train=None, y_train=None, individual_list=None, size=None,
                 crossover_rate=0.5, mutation_rate=0.015, maximize=True,
                 additional_parameters=None, evaluator=None):
        self.x_train = x_train
        self.y_train = y_train
        self.species = species
        self.maximize = maximize
        self.crossover_rate = crossover_rate
        self.mutation_rate = mutation_rate
        self.additional_parameters = dict(additional_parameters or {})
        self.evaluator = evaluator
        if individual_list is None and size is None:
            raise ValueError("Either pass a list of individuals or a population size for a random population.")
        if individual_list is None:
            self.individuals = [
                species(x_train, y_train, crossover_rate=crossover_rate, mutation_rate=mutation_rate,
                        **self.additional_parameters)
                for _ in range(size)
            ]
            self.population_size = size
            print("Initializing a random population. Size: {}".format(size))
        else:
            for ind in individual_list:
                if type(ind) is not species:
                    raise AssertionError("All individuals must be of species {}".format(species.__name__))
            self.individuals = individual_list
            self.population_size = len(individual_list)

    # ------------------------------------------------------------------ basic
    def add_individual(self, individual):
        if type(individual) is not self.species:
            raise AssertionError("Individual is not of species {}".format(self.species.__name__))
        self.individuals.append(individual)
        self.population_size += 1

    def get_species(self):
        return self.species

    def get_size(self):
        return self.population_size

    def get_data(self):
        return self.x_train, self.y_train

    def get_fitness_criteria(self):
        return self.maximize

    def __getitem__(self, item):
        return self.individuals[item]

    def __len__(self):
        return self.population_size

    def __iter__(self):
        return iter(self.individuals)

    # ------------------------------------------------------------- evaluation
    def pending(self):
        """Individuals whose fitness is not known yet (deduplicated by identity)."""
        seen, out = set(), []
        for ind in self.individuals:
            if not ind.get_fitness_status() and id(ind) not in seen:
                seen.add(id(ind))
                out.append(ind)
        return out

    def evaluate_pending(self):
        """Batch-evaluate pending individuals with the attached evaluator.
        Returns the number of fitness evaluations performed."""
        todo = self.pending()
        if not todo:
            return 0
        if self.evaluator is None:
            for ind in todo:
                ind.get_fitness()
            return len(todo)
        return self.evaluator.evaluate(todo)

    def get_fittest(self):
        """Max (or min) by fitness; ties resolve to the first individual.
        (reference: gentun/populations.py:55-58)"""
        if self.evaluator is not None:
            self.evaluate_pending()
        pick = max if self.maximize else min
        return pick(self.individuals, key=operator.methodcaller('get_fitness'))

    # ------------------------------------------------------------ derivation
    def empty_like(self, individual_list=None):
        """A population of the same class and evaluation strategy."""
        return Population(self.species, self.x_train, self.y_train,
                          individual_list=[] if individual_list is None else individual_list,
                          crossover_rate=self.crossover_rate, mutation_rate=self.mutation_rate,
                          maximize=self.maximize, additional_parameters=self.additional_parameters,
                          evaluator=self.evaluator)


class GridPopulation(Population):
    """Initial population from the Cartesian product of per-gene value lists.

    Genes missing from ``genes_grid`` take the genome default (spec[0]).
    Only tuple-spec genomes (XGBoost-style) are supported; the reference
    crashes with a TypeError for bit-string genomes, we raise
    a clear ValueError instead.
    (reference: gentun/populations.py:70-105)
    """

    def __init__(self, species, x_train=None, y_train=None, individual_list=None, genes_grid=None,
                 crossover_rate=0.5, mutation_rate=0.015, maximize=True,
                 additional_parameters=None, evaluator=None):
        additional_parameters = dict(additional_parameters or {})   # Q8: None -> {}
        if individual_list is None and genes_grid is None:
            raise ValueError("Either pass a list of individuals or a grid definition.")
        if genes_grid is not None:
            genome = species(None, None).get_genome()
            unknown = set(genes_grid) - set(genome)
            if unknown:
                raise ValueError("Some grid parameters do not belong to the species' genome: {}".format(
                    sorted(unknown)))
            grid = dict(genes_grid)
            for name, spec in genome.items():
                if name not in grid:
                    if not isinstance(spec, (tuple, list)):
                        raise ValueError("GridPopulation needs tuple gene specs (default, min, max, base); "
                                         "species {} uses {!r}".format(species.__name__, spec))
                    grid[name] = [spec[0]]
            names = list(grid)
            individual_list = [
                species(x_train, y_train, genes=dict(zip(names, combo)), crossover_rate=crossover_rate,
                        mutation_rate=mutation_rate, **additional_parameters)
                for combo in itertools.product(*(grid[n] for n in names))
            ]
            print("Initializing a grid population. Size: {}".format(len(individual_list)))
        super(GridPopulation, self).__init__(species, x_train, y_train, individual_list, None, crossover_rate,
                                             mutation_rate, maximize, additional_parameters, evaluator)

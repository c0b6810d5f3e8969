"""Abstract fitness model (reference: gentun/models/generic_models.py:7-18)."""


class GentunModel(object):
    """Holds the training data; ``cross_validate()`` returns the scalar fitness."""

    def __init__(self, x_train, y_train):
        self.x_train = x_train
        self.y_train = y_train

    def cross_validate(self):
        raise NotImplementedError("Use a subclass with a defined model.")

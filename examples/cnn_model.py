#!/usr/bin/env python
"""Single Genetic-CNN model (all-zero genes), 5-fold CV on MNIST-shaped data
(reference tests/test_keras_model.py:11-39). Runs the HIP executor on a GPU,
the PyTorch executor on the CPU."""
import _common

if __name__ == "__main__":
    from gentun import GeneticCnnModel

    x_train, y_train = _common.mnist_like()
    model = GeneticCnnModel(
        x_train, y_train,
        {'S_1': '000', 'S_2': '0000000000'},  # Genes to test
        (28, 28, 1),  # Shape of input data
        (20, 50),  # Number of kernels per layer
        ((5, 5), (5, 5)),  # Sizes of kernels per layer
        500,  # Number of units in Dense layer
        0.5,  # Dropout probability
        10,  # Number of classes to predict
        nfold=5,
        epochs=(20, 4, 1),
        learning_rate=(1e-3, 1e-4, 1e-5),
        batch_size=128
    )
    print(model.cross_validate())

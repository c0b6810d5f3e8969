#!/usr/bin/env python
"""Single Genetic-CNN model (all-zero genes), 5-fold CV on MNIST-shaped data
(reference tests/test_keras_model.py:11-39, with the ``nodes`` argument that
the reference script omits although GeneticCnnModel requires it,
gentun/models/keras_models.py:21-22). Runs the HIP executor on a GPU, the
PyTorch executor on the CPU."""
import _common

if __name__ == "__main__":
    from gentun import GeneticCnnModel

    x_train, y_train = _common.mnist_like()
    sched = _common.cnn_schedule()
    model = GeneticCnnModel(
        x_train, y_train,
        genes={'S_1': '000', 'S_2': '0000000000'},
        nodes=(3, 5),
        input_shape=(28, 28, 1),
        kernels_per_layer=(20, 50),
        kernel_sizes=((5, 5), (5, 5)),
        dense_units=500,
        dropout_probability=0.5,
        classes=10,
        nfold=sched['nfold'],
        epochs=sched['epochs'],
        learning_rate=sched['learning_rate'],
        batch_size=128,
    )
    print(model.cross_validate())

"""Callback hook protocol the training loops call (reference callbacks.py:1-30).

Only the base class is part of the hot path's API; the reference's WandB / TensorBoard
loggers (callbacks.py:35-70) are a logging side channel and are out of scope here -- any
object implementing these hooks can be passed to the loops.
"""


class Callback:
    def on_train_begin(self, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_batch_end(self, batch, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_validation_batch_end(self, batch, logs=None):
        pass

    def on_validation_begin(self, logs=None):
        pass

    def on_validation_end(self, logs=None, data=None):
        pass

    def on_test_begin(self, logs=None):
        pass

    def on_test_end(self, logs=None):
        pass

"""Utilities: meters, flatten/unflatten, stochastic quantisation, metrics writers."""
from .meters import Average, EMAverage, Accuracy
from .flatten import flatten, flatten_torch_tensor, unflatten, unflatten_torch_tensor
from .quantize import quantize_tensor
from .logging import MetricsWriter, PhaseTimer

__all__ = ['Average', 'EMAverage', 'Accuracy', 'flatten',
           'flatten_torch_tensor', 'unflatten', 'unflatten_torch_tensor', 'quantize_tensor',
           'MetricsWriter', 'PhaseTimer']

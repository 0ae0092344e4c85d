"""Train / validation / test split algorithms for the downstream tasks
(reference: shallow_encoders/split/__init__.py)."""
from shallow_encoders.split.core import (
    SplitAlgorithm,
    TrainTestRatioSplit,
    TrainValTestRatioSplit,
    TrainValTestStratifiedNSamplesSplit,
)

__all__ = ['SplitAlgorithm', 'TrainTestRatioSplit', 'TrainValTestRatioSplit',
           'TrainValTestStratifiedNSamplesSplit']

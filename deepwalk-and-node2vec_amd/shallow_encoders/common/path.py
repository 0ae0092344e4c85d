"""Project paths (shallow_encoders/common/path.py:8-11 of the reference): ROOT is the
directory that holds the ``shallow_encoders`` package, ``configs/`` and ``tools/``."""
import os
from pathlib import Path

ROOT_PATH = str(Path(__file__).parent.parent.parent)
CONFIG_PATH = os.path.join(ROOT_PATH, 'configs')
RUNS_PATH = os.path.join(ROOT_PATH, 'runs')
ASSETS_PATH = os.path.join(ROOT_PATH, 'assets')

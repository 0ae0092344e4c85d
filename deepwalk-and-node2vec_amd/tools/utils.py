"""Tool helpers (reference: tools/utils.py:19-43)."""
import os
from datetime import datetime
from pathlib import Path
from typing import Any, Dict

import yaml

from shallow_encoders.common.path import RUNS_PATH
from shallow_encoders.config_parser import config_from_dict, print_config_tree
from shallow_encoders.config_parser.core import GlobalConfig
from tools.conventions import DATETIME_FORMAT, get_run_history_experiment_path


def setup_pipeline(cfg: Dict[str, Any], task: str) -> GlobalConfig:
    """Print the config tree, save it to the run history, return the typed config.

    Like the reference, the run-history root is the TOP-LEVEL ``output_dir`` key (default
    runs/), not ``path.output_dir`` (tools/utils.py:35)."""
    print_config_tree(cfg)
    output_dir = cfg.get('output_dir', RUNS_PATH)
    config_dirpath = get_run_history_experiment_path(output_dir, cfg['datamodule']['dataset_name'],
                                                     cfg['train']['experiment'])
    dt = datetime.now().strftime(DATETIME_FORMAT)
    Path(config_dirpath).mkdir(parents=True, exist_ok=True)
    with open(os.path.join(config_dirpath, f'{task}_{dt}.yaml'), 'w', encoding='utf-8') as f:
        f.write(yaml.safe_dump(cfg, sort_keys=False))
    return config_from_dict(cfg)

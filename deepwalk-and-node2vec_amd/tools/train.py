"""Train a skip-gram model on graph random walks (reference: tools/train.py:21-88).

    python tools/train.py --config-name=sge_sg_karate_club [key.sub=value ...]

Same configs, run-history dump, output layout and checkpoint names as the reference; the PL
Trainer is replaced by shallow_encoders.word2vec.fit (walks and SGNS on the MI355X).
"""
import argparse
import logging
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from shallow_encoders.common.path import CONFIG_PATH  # noqa: E402
from shallow_encoders.config_parser import load_config_dict  # noqa: E402
from shallow_encoders.word2vec.fit import fit  # noqa: E402
from tools import conventions  # noqa: E402
from tools.utils import setup_pipeline  # noqa: E402

logger = logging.getLogger('Trainer')


def check_train_experiment_history(output_dir: str, dataset_name: str, experiment: str) -> None:
    """Offer to delete an experiment's previous checkpoints / logs (tools/train.py:21-42).
    Non-interactive runs keep the history."""
    dirpaths = [conventions.get_tb_logs_experiment_path(output_dir, dataset_name, experiment),
                conventions.get_checkpoints_experiment_path(output_dir, dataset_name, experiment)]
    if any(os.path.exists(p) for p in dirpaths):
        logger.warning(f'Experiment "{experiment}" already has some history.')
        if sys.stdin.isatty():
            response = input(f'Delete "{experiment}" history? [yes/no]   ')
            if response.lower() == 'yes':
                for p in dirpaths:
                    if os.path.exists(p):
                        shutil.rmtree(p)


def parse_args(argv):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument('--config-name', '-cn', default='sge_sg_karate_club')
    ap.add_argument('--config-path', '-cp', default=CONFIG_PATH)
    ap.add_argument('overrides', nargs='*', help='key.sub=value overrides')
    return ap.parse_args(argv)


def main(argv=None) -> dict:
    args = parse_args(sys.argv[1:] if argv is None else argv)
    raw = load_config_dict(args.config_name, args.config_path, args.overrides)
    cfg = setup_pipeline(raw, task='train')
    check_train_experiment_history(cfg.path.output_dir, cfg.datamodule.dataset_name,
                                   cfg.train.experiment)
    import torch
    torch.manual_seed(cfg.train.seed)
    dataset = cfg.datamodule.instantiate_dataset()
    dataloader = cfg.datamodule.instantiate_dataloader(dataset=dataset)
    trainer = cfg.instantiate_trainer(dataset=dataset)
    out = cfg.path.output_dir
    ds, exp = cfg.datamodule.dataset_name, cfg.train.experiment
    return fit(trainer, dataloader, cfg.train.max_epochs,
               checkpoint_dir=conventions.get_checkpoints_experiment_path(out, ds, exp),
               log_dir=conventions.get_tb_logs_experiment_path(out, ds, exp))


if __name__ == '__main__':
    main()

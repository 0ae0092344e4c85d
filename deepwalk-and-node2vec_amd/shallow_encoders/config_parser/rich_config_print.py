"""Rich tree print of a config (reference: config_parser/rich_config_print.py:16-68)."""
import dataclasses
import logging
from typing import Sequence

import yaml

logger = logging.getLogger('RichTree')


def print_config_tree(cfg, print_order: Sequence[str] = ('datamodule', 'train', 'model'),
                      resolve: bool = False) -> None:
    """Print each top-level section as YAML under a rich tree (plain text without rich)."""
    data = dataclasses.asdict(cfg) if dataclasses.is_dataclass(cfg) else dict(cfg)
    queue = [f for f in print_order if f in data]
    for f in print_order:
        if f not in data:
            logger.warning(f'Field "{f}" not found in config. Skipping "{f}" config printing...')
    queue += [f for f in data if f not in queue]
    try:
        import rich
        import rich.syntax
        import rich.tree
    except ImportError:  # pragma: no cover
        for f in queue:
            print(f'{f}:\n{yaml.safe_dump(data[f], sort_keys=False)}')
        return
    style = 'dim'
    tree = rich.tree.Tree('CONFIG', style=style, guide_style=style)
    for f in queue:
        branch = tree.add(f, style=style, guide_style=style)
        content = data[f]
        text = yaml.safe_dump(content, sort_keys=False) if isinstance(content, dict) else str(content)
        branch.add(rich.syntax.Syntax(text, 'yaml'))
    rich.print(tree)

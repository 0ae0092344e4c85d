from shallow_encoders.config_parser.core import (GlobalConfig, instantiate, load_config,
                                                 load_config_dict, config_from_dict)
from shallow_encoders.config_parser.rich_config_print import print_config_tree

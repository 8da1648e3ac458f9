from .cfgnode import CfgNode, load_cfg
from .defaults import CFG, get_cfg, dump_cfg, METHOD_NODES

__all__ = ["CfgNode", "load_cfg", "CFG", "get_cfg", "dump_cfg", "METHOD_NODES"]

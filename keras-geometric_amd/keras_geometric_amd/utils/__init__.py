from .data import GraphData, batch_graphs
from .io import load_graphs, save_graphs
from .main import add_self_loops, compute_gcn_normalization

__all__ = ["GraphData", "add_self_loops", "batch_graphs", "compute_gcn_normalization", "load_graphs", "save_graphs"]

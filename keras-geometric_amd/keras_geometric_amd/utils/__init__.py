from .main import add_self_loops, compute_gcn_normalization

__all__ = ["add_self_loops", "compute_gcn_normalization"]

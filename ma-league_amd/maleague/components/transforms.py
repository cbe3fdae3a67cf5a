"""Preprocess transforms (API of src/marl/components/transforms.py:12-22)."""
import torch


class Transform:
    def transform(self, tensor):
        raise NotImplementedError

    def infer_output_info(self, vshape_in, dtype_in):
        raise NotImplementedError


class OneHot(Transform):
    """Integer index [..., 1] -> float one-hot [..., out_dim]."""

    def __init__(self, out_dim):
        self.out_dim = out_dim

    def transform(self, tensor):
        out = torch.zeros(*tensor.shape[:-1], self.out_dim, dtype=tensor.dtype, device=tensor.device)
        out.scatter_(-1, tensor.long(), 1)
        return out.float()

    def infer_output_info(self, vshape_in, dtype_in):
        return (self.out_dim,), torch.float32

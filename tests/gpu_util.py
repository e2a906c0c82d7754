"""Helpers shared by GPU tests: numpy <-> device tensors in the fixtures' representation."""
import numpy as np
import torch


def to_dev(a, device="cuda:0"):
    """uint16 bits -> bfloat16; float16 / float32 map to torch.float16 / torch.float32."""
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        return torch.from_numpy(a.view(np.int16)).view(torch.bfloat16).to(device)
    return torch.from_numpy(a).to(device)


def to_np(t):
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def kind_of(tin, tout):
    if tout is tin:
        return "same"
    if tout.untyped_storage().data_ptr() == tin.untyped_storage().data_ptr():
        return "view"
    return "new"

"""CompressFn protocol (reference: kvcompress/methods/base.py:12-50)."""
from typing import List, Protocol, Tuple, runtime_checkable

import torch

from ..utils import normalize_kv_cache  # noqa: F401  (re-exported like the reference)


@runtime_checkable
class CompressFn(Protocol):
    def __call__(self, past_key_values, **kwargs) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        ...

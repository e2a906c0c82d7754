"""CPU baseline port -- TEST/BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

The reference's fix_size_l2 keep_low path (kvcompress/methods/fix_size_l2.py:99-150) restated as
the same torch CPU op sequence -- norm -> argsort -> [:keep] -> sort -> gather (-> cat) -- so the
GPU box's host cores can be timed on exactly the work the reference does.  Its outputs are the
reference's (tests/test_oracle_golden.py pins the numpy oracle; this port is checked against it
in tests/test_torch_port.py).
"""
import torch


def fix_size_l2_layer(keys, values, fix_kv_size=512, keep_ratio=0.0):
    seq_len = keys.size(2)
    B, H, S, D = keys.shape
    P = min(int(fix_kv_size * keep_ratio), seq_len)
    Z = seq_len - P
    keep = fix_kv_size - P
    ek, ev = keys[:, :, :Z, :], values[:, :, :Z, :]
    order = torch.norm(ek, p=2, dim=-1).argsort(dim=-1)
    idx, _ = torch.sort(order[:, :, :keep], dim=-1)
    e = idx.unsqueeze(-1).expand(B, H, keep, D)
    kk, kv = torch.gather(ek, 2, e), torch.gather(ev, 2, e)
    if P > 0:
        return torch.cat([kk, keys[:, :, -P:, :]], dim=2), torch.cat([kv, values[:, :, -P:, :]], dim=2)
    return kk, kv

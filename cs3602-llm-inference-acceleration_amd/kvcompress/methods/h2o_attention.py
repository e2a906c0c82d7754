"""h2o_attention (reference: kvcompress/methods/h2o_attention.py) -- not part of this engine.

It selects heavy hitters from accumulated attention probabilities (output_attentions=True),
not from key norms, so it is outside the key-norm hot path this MI355X engine implements
(SURVEY §8f rank 4).  The name stays registered so list_methods() matches the reference;
calling it raises.
"""


class H2OAttentionManager:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            "h2o_attention (attention-score heavy hitters) is not implemented by the MI355X "
            "key-norm engine (SURVEY §8f rank 4)")


def create_h2o_manager_from_model(*args, **kwargs):
    return H2OAttentionManager(*args, **kwargs)


def h2o_attention_compress(past_key_values, *args, **kwargs):
    raise NotImplementedError(
        "h2o_attention (attention-score heavy hitters) is not implemented by the MI355X "
        "key-norm engine (SURVEY §8f rank 4); use h2o_l2")


__all__ = ["h2o_attention_compress", "H2OAttentionManager", "create_h2o_manager_from_model"]

"""Parameter layouts (names + shapes in `parameters()` order) of the models the benchmark and
the tests use. No weights, no network: shapes only, so arenas of the named sizes can be built
with synthetic values on the device.

  tiny_llama       EDT_LM/train/init_weights.py:46-71   P =     6,570,560  T =  39
  gpt2_small       GPT-2 small (125M class)             P =   124,439,808  T = 148
  gpt_1p3b         GPT 2048 x 24 (1.3B class)           P = 1,315,723,264  T = 292
  qwen2p5_7b_body  Qwen2.5-7B `model.model`, EDT_EVOMERGE/train/crossover.py:142
                                                        P = 7,070,619,136  T = 338
  ivy_policy       EDT_RL/train/model.py:25-45 Ivy transformer (hidden 32, 4 layers), RL SLERP keys
"""
from __future__ import annotations

from .params import ParamLayout


def _gpt(vocab: int, n_ctx: int, d: int, layers: int) -> ParamLayout:
    names, shapes = ["wte.weight", "wpe.weight"], [(vocab, d), (n_ctx, d)]
    for i in range(layers):
        p = f"h.{i}."
        for n, s in (("ln_1.weight", (d,)), ("ln_1.bias", (d,)), ("attn.c_attn.weight", (d, 3 * d)),
                     ("attn.c_attn.bias", (3 * d,)), ("attn.c_proj.weight", (d, d)), ("attn.c_proj.bias", (d,)),
                     ("ln_2.weight", (d,)), ("ln_2.bias", (d,)), ("mlp.c_fc.weight", (d, 4 * d)),
                     ("mlp.c_fc.bias", (4 * d,)), ("mlp.c_proj.weight", (4 * d, d)), ("mlp.c_proj.bias", (d,))):
            names.append(p + n)
            shapes.append(s)
    names += ["ln_f.weight", "ln_f.bias"]
    shapes += [(d,), (d,)]
    return ParamLayout(shapes, names)


def _llama(vocab, d, inter, layers, heads, kv, head_dim, bias=False, lm_head=True, prefix="model.") -> ParamLayout:
    names, shapes = [prefix + "embed_tokens.weight"], [(vocab, d)]
    for i in range(layers):
        p = f"{prefix}layers.{i}."
        items = [("self_attn.q_proj.weight", (heads * head_dim, d))]
        if bias:
            items.append(("self_attn.q_proj.bias", (heads * head_dim,)))
        items.append(("self_attn.k_proj.weight", (kv * head_dim, d)))
        if bias:
            items.append(("self_attn.k_proj.bias", (kv * head_dim,)))
        items.append(("self_attn.v_proj.weight", (kv * head_dim, d)))
        if bias:
            items.append(("self_attn.v_proj.bias", (kv * head_dim,)))
        items += [("self_attn.o_proj.weight", (d, heads * head_dim)), ("mlp.gate_proj.weight", (inter, d)),
                  ("mlp.up_proj.weight", (inter, d)), ("mlp.down_proj.weight", (d, inter)),
                  ("input_layernorm.weight", (d,)), ("post_attention_layernorm.weight", (d,))]
        for n, s in items:
            names.append(p + n)
            shapes.append(s)
    names.append(prefix + "norm.weight")
    shapes.append((d,))
    if lm_head:
        names.append("lm_head.weight")
        shapes.append((vocab, d))
    return ParamLayout(shapes, names)


def tiny_llama() -> ParamLayout:
    return _llama(49152, 64, 256, 4, 4, 1, 32)


def gpt2_small() -> ParamLayout:
    return _gpt(50257, 1024, 768, 12)


def gpt_1p3b() -> ParamLayout:
    return _gpt(50257, 2048, 2048, 24)


def qwen2p5_7b_body() -> ParamLayout:
    return _llama(152064, 3584, 18944, 28, 28, 4, 128, bias=True, lm_head=False, prefix="")


def ivy_policy(obs: int = 30, out: int = 40) -> ParamLayout:
    """Ivy4RL-shaped state dict (hidden 32, 4 layers, 4 heads / 2 kv) with a head."""
    lay = _llama(0, 32, 128, 4, 4, 2, 8, bias=True, lm_head=False, prefix="")
    names = ["obs_proj.weight"] + lay.names[1:] + ["rl_head.weight"]
    shapes = [(32, obs)] + lay.shapes[1:] + [(out, 32)]
    return ParamLayout(shapes, names)


LAYOUTS = {
    "tiny_llama": tiny_llama,
    "gpt2_small": gpt2_small,
    "gpt_1p3b": gpt_1p3b,
    "qwen2p5_7b_body": qwen2p5_7b_body,
    "ivy_policy": ivy_policy,
}

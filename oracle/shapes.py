"""State-dict {key: shape} maps of the reference's decoder modules (checkpoint key names,
utils/utils.py:209-216)."""


def lstm_decoder_shapes(E, A, D, Em, V):
    """DecoderWithAttention(attention_dim=A, embed_dim=Em, decoder_dim=D, vocab_size=V, encoder_dim=E)
    (models/decoder.py:35-57)."""
    return {
        "attention.encoder_att.weight": (A, E), "attention.encoder_att.bias": (A,),
        "attention.decoder_att.weight": (A, D), "attention.decoder_att.bias": (A,),
        "attention.full_att.weight": (1, A), "attention.full_att.bias": (1,),
        "embedding.weight": (V, Em),
        "decode_step.weight_ih": (4 * D, Em + E), "decode_step.weight_hh": (4 * D, D),
        "decode_step.bias_ih": (4 * D,), "decode_step.bias_hh": (4 * D,),
        "init_h.weight": (D, E), "init_h.bias": (D,),
        "init_c.weight": (D, E), "init_c.bias": (D,),
        "f_beta.weight": (E, D), "f_beta.bias": (E,),
        "fc.weight": (V, D), "fc.bias": (V,),
    }


def transformer_decoder_shapes(E, d, ff, V, layers):
    """TransformerDecoder(embed_dim=d, decoder_dim=ff, vocab_size=V, encoder_dim=E, num_layers=layers)
    (models/transformerDecoder.py:53-86); ``pos_encoding.pe`` is a buffer, not listed."""
    s = {"embedding.weight": (V, d), "fc_out.weight": (V, d), "fc_out.bias": (V,)}
    if E != d:
        s.update({"encoder_proj.weight": (d, E), "encoder_proj.bias": (d,)})
    for i in range(layers):
        p = f"transformer_decoder.layers.{i}."
        for a in ("self_attn", "multihead_attn"):
            s.update({p + a + ".in_proj_weight": (3 * d, d), p + a + ".in_proj_bias": (3 * d,),
                      p + a + ".out_proj.weight": (d, d), p + a + ".out_proj.bias": (d,)})
        s.update({p + "linear1.weight": (ff, d), p + "linear1.bias": (ff,),
                  p + "linear2.weight": (d, ff), p + "linear2.bias": (d,)})
        for n in ("norm1", "norm2", "norm3"):
            s.update({p + n + ".weight": (d,), p + n + ".bias": (d,)})
    return s

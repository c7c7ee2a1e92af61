"""World-size-2 gloo run of the trainer's DDP path on CPU (trainMultiGPU.py:339-420): rank-0
weight broadcast, SUM all-reduce of the flat gradient with the 1/world mean folded into the
Adam step, fused metric all-reduce -- checked against the reference's own 2-rank run
(tests/golden/ddp2_lstm, produced by trainMultiGPU.trainWithTeacherForcing under gloo DDP)."""
import ddp_util


def test_trainer_ddp2_matches_reference_trainMultiGPU(tmp_path):
    ddp_util.check(ddp_util.run("oracle", tmp_path))


def test_trainer_ddp2_unbucketed_matches_reference(tmp_path):
    """The same run with the bucketed all-reduce switched off (one collective after backward)."""
    ddp_util.check(ddp_util.run("oracle", tmp_path, bucketed=False))


def test_trainer_ddp2_transformer_finetuned_encoder_matches_oracle_average(tmp_path):
    """Transformer decoder + a trainable encoder over 2 gloo ranks (trainMultiGPU.py:233-235,
    256, 384-394): rank 0's weights broadcast, the decoder's gradients reduced as one bucket
    before the encoder backward, the encoder's after it, clip, both Adams -- equal to the
    oracle's single-process averaged step; with and without the bucket."""
    import ddp_ft_util
    ddp_ft_util.check(ddp_ft_util.run(tmp_path / "b", bucketed=True))
    ddp_ft_util.check(ddp_ft_util.run(tmp_path / "u", bucketed=False))

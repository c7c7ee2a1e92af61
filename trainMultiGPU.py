"""Multi-GPU (one process per GPU) teacher-forced training entry point, trainMultiGPU.py's
counterpart: SLURM variables (trainMultiGPU.py:144-146) or torchrun's RANK / WORLD_SIZE /
LOCAL_RANK, backend "nccl" (= RCCL over xGMI), DDP-equivalent gradient averaging inside
``TeacherForcedTrainer`` (one all-reduce of the flat gradient buffer per step) and the
``reduceLossAndTokens`` metric reduction (:96-108).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 trainMultiGPU.py \
        --teacherForcing --encoder base --batchSize 32
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import train  # noqa: E402  (model construction, CLI and the epoch loop are shared)


def setup_distributed():
    """trainMultiGPU.py:144-160 (SLURM) or torchrun environment."""
    if "SLURM_PROCID" in os.environ and "RANK" not in os.environ:
        rank, world, local = (int(os.environ[k]) for k in ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"))
    else:
        rank, world, local = (int(os.environ.get(k, d)) for k, d in (("RANK", 0), ("WORLD_SIZE", 1),
                                                                       ("LOCAL_RANK", 0)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    torch.cuda.set_device(local)
    device = torch.device(f"cuda:{local}")
    dist.init_process_group("nccl", init_method="env://", world_size=world, rank=rank, device_id=device)
    return rank, local, world, device


def main(argv=None):
    args = train.parse(argv)
    if not args.teacherForcing:
        raise NotImplementedError("non-teacher-forced training is outside the accelerated path (SURVEY.md §8f)")
    rank, local, world, device = setup_distributed()
    torch.manual_seed(42 + rank)
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    encoder, decoder, ck = train.build_models(args, device)
    trainer = TeacherForcedTrainer(encoder, decoder, lstm=args.lstmDecoder, decoder_lr=train.decoderLr,
                                   encoder_lr=args.encoderLr, grad_clip=train.gradClip, alphaC=train.alphaC,
                                   graph=True)
    log = print if rank == 0 else (lambda *a, **k: None)
    # trainMultiGPU.py: encoder fine-tuned (and DDP-averaged) from epoch 20; rank 0 checkpoints
    train.run_epochs(args, encoder, decoder, trainer, ck, device, rank=rank, log=log, world=world)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

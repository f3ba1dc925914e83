"""Training entry point with the reference CLI (moegan/train_model.py:38-146) on the MI355X path.

Same flags and defaults; data are the preprocessed MS-COCO arrays (images [N,3,64,64] in [-1,1],
CLIP text embeddings [N,512]) read memory-mapped.  Extra flags select the MoE configuration and the
compute dtype.  Data parallel: launch one process per GPU with torch.distributed.run; each rank reads
a disjoint shard of every epoch (DistributedSampler) and gradients are all-reduced over RCCL.
"""
import argparse
import os
import sys

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BATCH_SIZE = 2
NUM_EPOCHS = 10
LEARNING_RATE = 0.0002
BETA1 = 0.5
BETA2 = 0.999
R1_GAMMA = 10.0
CLIP_WEIGHT_64 = 0.1
CLIP_WEIGHT_32 = 0.05
KL_WEIGHT = 0.001
BALANCE_WEIGHT = 0.01


class ShardSampler(torch.utils.data.Sampler):
    """Rank ``rank``'s share of ``n`` validation samples, indices rank::world, with no padding: the all-reduced
    validation sums then count every sample exactly once, as the single-process reference does
    (t2i_moe_gan.py:1432-1473).  (DistributedSampler(drop_last=False) repeats samples to even out the shards.)"""

    def __init__(self, n, rank, world):
        self.idx = list(range(rank, n, world))

    def __iter__(self):
        return iter(self.idx)

    def __len__(self):
        return len(self.idx)


class ProcessedMSCOCODataset(Dataset):
    """(image, text_embedding) pairs from two .npy files (data_processing_pipeline.py:425-470), memory-mapped."""

    def __init__(self, images_file, text_embeddings_file):
        self.images = np.load(images_file, mmap_mode="r")
        self.text_embeddings = np.load(text_embeddings_file, mmap_mode="r")
        assert len(self.images) == len(self.text_embeddings), "Images and text embeddings count mismatch"

    def __len__(self):
        return len(self.images)

    def __getitem__(self, idx):
        return torch.from_numpy(np.array(self.images[idx])), torch.from_numpy(np.array(self.text_embeddings[idx]))


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Train Aurora GAN-MoE (MI355X)")
    p.add_argument("--data_dir", type=str, default="../data_processing/processed_data")
    p.add_argument("--train_images", type=str, default="mscoco_train_images.npy")
    p.add_argument("--train_embeddings", type=str, default="mscoco_train_text_embeddings.npy")
    p.add_argument("--val_images", type=str, default="mscoco_validation_images.npy")
    p.add_argument("--val_embeddings", type=str, default="mscoco_validation_text_embeddings.npy")
    p.add_argument("--batch_size", type=int, default=BATCH_SIZE)
    p.add_argument("--epochs", type=int, default=NUM_EPOCHS)
    p.add_argument("--lr", type=float, default=LEARNING_RATE)
    p.add_argument("--beta1", type=float, default=BETA1)
    p.add_argument("--beta2", type=float, default=BETA2)
    p.add_argument("--save_dir", type=str, default="./aurora_checkpoints_v2")
    p.add_argument("--log_interval", type=int, default=50)
    p.add_argument("--save_interval", type=int, default=1000)
    p.add_argument("--r1_gamma", type=float, default=R1_GAMMA)
    p.add_argument("--clip_weight_64", type=float, default=CLIP_WEIGHT_64)
    p.add_argument("--clip_weight_32", type=float, default=CLIP_WEIGHT_32)
    p.add_argument("--kl_weight", type=float, default=KL_WEIGHT)
    p.add_argument("--balance_weight", type=float, default=BALANCE_WEIGHT)
    # MI355X extras
    p.add_argument("--num_experts", type=int, default=4)
    p.add_argument("--topk", type=int, default=None, help="sparse top-k routing (default: dense soft combine)")
    p.add_argument("--dtype", choices=["fp32", "bf16"], default="bf16")
    p.add_argument("--gradient_accumulation_steps", type=int, default=8)
    p.add_argument("--resume", type=str, default=None, help="resume checkpoint (t2i_moe_gan.py:1484-1491 layout)")
    p.add_argument("--save_every_epoch", action="store_true", help="write a resume checkpoint after every epoch")
    p.add_argument("--max_resolution", type=int, default=16, choices=[16, 32, 64, 128],
                   help="generator output size: 16 = the reference; 32/64/128 = the progressive extension")
    p.add_argument("--clip_weights", type=str, default=None,
                   help="local OpenAI CLIP state_dict / safetensors: enables the (gradient-free) CLIP loss terms")
    p.add_argument("--hyperparameters", type=str, default=None,
                   help="SageMaker-style hyperparameters.json (string values, sagemaker_train.py:85-102); batch_size "
                        "and the train_aurora_gan keys override the flags above, other keys are reported as unused")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    import t2i_moe_gan as M
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    pg = None
    device = M.DEVICE
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", 0))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        dist.init_process_group("nccl")
        pg = dist.group.WORLD
    hp = {}
    if args.hyperparameters:  # read before the DataLoaders: batch_size sizes them (sagemaker_train.py:233, :248)
        from moegan_mi.hparams import load_sagemaker_hyperparameters
        hp = load_sagemaker_hyperparameters(args.hyperparameters)
        if "batch_size" in hp:
            args.batch_size = int(hp["batch_size"])
    if rank == 0:
        print(f"Using device: {device}")
        print(f"Training args: {args}")
    os.makedirs(args.save_dir, exist_ok=True)
    tr_i = os.path.join(args.data_dir, args.train_images)
    tr_e = os.path.join(args.data_dir, args.train_embeddings)
    va_i = os.path.join(args.data_dir, args.val_images)
    va_e = os.path.join(args.data_dir, args.val_embeddings)
    if not os.path.exists(tr_i) or not os.path.exists(tr_e):
        print(f"Error: Training data not found at {tr_i} or {tr_e}")
        sys.exit(1)
    val_ds = ProcessedMSCOCODataset(va_i, va_e) if os.path.exists(va_i) and os.path.exists(va_e) else None
    if val_ds is None:
        print(f"Warning: Validation data not found at {va_i} or {va_e}. Skipping validation.")
    train_ds = ProcessedMSCOCODataset(tr_i, tr_e)
    sampler = None
    if world > 1:
        from torch.utils.data.distributed import DistributedSampler
        sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True, drop_last=True)
    workers = max(1, min(8, (os.cpu_count() or 2) // 2))
    train_dl = DataLoader(train_ds, batch_size=args.batch_size, shuffle=sampler is None, sampler=sampler,
                          num_workers=workers, pin_memory=True, drop_last=True)
    val_dl = None
    if val_ds is not None:  # every rank validates its shard; the sums are all-reduced inside the loop
        vs = ShardSampler(len(val_ds), rank, world) if world > 1 else None
        val_dl = DataLoader(val_ds, batch_size=args.batch_size, shuffle=False, sampler=vs, num_workers=workers,
                            pin_memory=True)
    kw = dict(num_epochs=args.epochs, lr=args.lr, beta1=args.beta1, beta2=args.beta2, r1_gamma=args.r1_gamma,
              clip_weight_16=args.clip_weight_64, clip_weight_8=args.clip_weight_32, kl_weight=args.kl_weight,
              balance_weight=args.balance_weight, log_interval=args.log_interval, save_interval=args.save_interval,
              gradient_accumulation_steps=args.gradient_accumulation_steps)
    if hp:
        from moegan_mi.hparams import unapplied_keys, given_train_kwargs
        kw.update(given_train_kwargs(hp))
        ignored = unapplied_keys(hp)
        if ignored and rank == 0:
            print(f"Warning: hyperparameters not used by training: {', '.join(sorted(ignored))}")
    if args.clip_weights:
        M.load_clip_weights(args.clip_weights, device)
    kw.setdefault("max_resolution", args.max_resolution)
    G, D = M.train_aurora_gan(train_dl, val_dataloader=val_dl, device=device, save_dir=args.save_dir,
                              num_experts=args.num_experts, topk=args.topk, dtype=args.dtype, process_group=pg,
                              resume_from=args.resume, save_every_epoch=args.save_every_epoch, **kw)
    if rank == 0:
        torch.save({"generator": G.state_dict(), "discriminator": D.state_dict()},
                   os.path.join(args.save_dir, "aurora_final.pt"))
        print("Training complete.")


if __name__ == "__main__":
    main()

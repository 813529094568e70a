"""The reference's per-folder CLIs on libvclip: `<folder>/main.py` (train + test evaluation) and
`<folder>/inference.py` (one video), same flags, same outputs.

  vivit_transformer/main.py          vivit_main        (train: the HIP train step, §8 a16)
  vivit_transformer/inference.py     vivit_inference
  timesformer/main.py, inference.py  timesformer_main / timesformer_inference
  videoswintransformer/...           swin_main / swin_inference
  resnet50-3d-video/...              resnet3d_main / resnet3d_inference

Launchers with the reference's folder layout live in `cli/<folder>/{main,inference}.py`.
Sampling is the bit-exact host sampler of each folder (vclip_amd.sampling); decode is host work
(vclip_amd.video_io); preprocessing and the model run on the GPU.  Outputs follow the reference:
`<log_dir>/<prefix>-YYYYmmdd_HHMMSS/` with `experiment.log`, `test_metrics_<method>.json`
(evaluator.py:99-120, metric keys of :257-401), best checkpoint dicts (trainer.py:291-305), and
`inference_results/<video>_result.json` (vivit_transformer/inference.py:225-248).
Only ViViT has a GPU backward; the other families' main.py evaluates a
checkpoint (`--skip_train` / `--checkpoint_path`, as resnet50-3d-video/main.py:53-56 offers) and
refuses to train rather than fall back to a CPU path.
"""
from __future__ import annotations

import argparse
import json
import logging
import random
import time
from datetime import datetime
from pathlib import Path

import numpy as np
import torch

from . import sampling, video_io

SAMPLING = ["random", "uniform", "random_window"]


# ------------------------------------------------------------------------- logging / bookkeeping
class ExperimentLogger:
    """Timestamped experiment dir with file + console handlers (vivit utils/logger.py:8-41)."""

    def __init__(self, log_dir, prefix="vivit-classifier"):
        self.exp_dir = Path(log_dir) / f"{prefix}-{datetime.now().strftime('%Y%m%d_%H%M%S')}"
        self.exp_dir.mkdir(parents=True, exist_ok=True)
        self.logger = logging.getLogger(f"{prefix}-{id(self)}")
        self.logger.setLevel(logging.INFO)
        self.logger.propagate = False
        fmt = logging.Formatter("%(asctime)s - %(levelname)s - %(message)s")
        for h in (logging.FileHandler(self.exp_dir / "experiment.log"), logging.StreamHandler()):
            h.setFormatter(fmt)
            self.logger.addHandler(h)

    def get_logger(self):
        return self.logger

    def get_experiment_dir(self):
        return self.exp_dir


def split_dir(root, mode):
    """The reference's data-dir resolution (vivit dataset.py:23-31)."""
    root = Path(root)
    if not (root / "dataset").exists():
        if (root / mode).exists():
            return root / mode
        return root / "dataset" / mode
    return root / "dataset" / mode


def scan_split(root, mode, logger):
    """(video paths, labels, class labels): class folders sorted by name (dataset.py:74-112)."""
    d = split_dir(root, mode)
    if not d.exists():
        raise FileNotFoundError(f"Data directory not found: {d}")
    classes = sorted(p.name for p in d.iterdir() if p.is_dir())
    paths, labels = [], []
    for ci, c in enumerate(classes):
        vids = video_io.list_videos(d / c)
        logger.info(f"Found {len(vids)} valid videos in class '{c}'")
        paths += vids
        labels += [ci] * len(vids)
    logger.info(f"Total videos for {mode}: {len(paths)}")
    return paths, labels, classes


def compute_metrics(labels, preds, probs, class_names):
    """evaluator.py:257-401 (binary: accuracy, confusion matrix, f1 / precision / recall,
    specificity, auroc + ROC / PR curves, optimal / best-F1 thresholds)."""
    from sklearn.metrics import (accuracy_score, average_precision_score, confusion_matrix, f1_score,
                                 precision_recall_curve, precision_score, recall_score, roc_auc_score, roc_curve)
    labels, preds, probs = np.asarray(labels), np.asarray(preds), np.asarray(probs)
    m = {}
    if len(labels) == 0:
        return dict(accuracy=0.0, f1_score=0.0, auroc=0.0, confusion_matrix=[])
    m["accuracy"] = float(accuracy_score(labels, preds))
    cm = confusion_matrix(labels, preds, labels=list(range(len(class_names))))
    m["confusion_matrix"] = cm.tolist()
    if len(class_names) == 2:
        m["f1_score"] = float(f1_score(labels, preds, zero_division=0))
        m["precision"] = float(precision_score(labels, preds, zero_division=0))
        m["recall"] = float(recall_score(labels, preds, zero_division=0))
        tn, fp = cm[0, 0], cm[0, 1]
        m["specificity"] = float(tn / (tn + fp)) if tn + fp > 0 else 0.0
        if len(np.unique(labels)) > 1:
            m["auroc"] = float(roc_auc_score(labels, probs[:, 1]))
            fpr, tpr, thr = roc_curve(labels, probs[:, 1])
            m["roc_curve"] = {"fpr": fpr.tolist(), "tpr": tpr.tolist(), "thresholds": thr.tolist()}
            m["optimal_threshold"] = float(thr[int(np.argmax(tpr - fpr))])
            pr, rc, pthr = precision_recall_curve(labels, probs[:, 1])
            m["pr_curve"] = {"precision": pr.tolist(), "recall": rc.tolist(), "thresholds": pthr.tolist()}
            m["average_precision"] = float(average_precision_score(labels, probs[:, 1]))
            f1s = [2 * p * r / (p + r) if p + r > 0 else 0.0 for p, r in zip(pr[:-1], rc[:-1])]
            if f1s:
                m["best_f1_threshold"] = float(pthr[int(np.argmax(f1s))])
        else:
            m["auroc"] = 0.0
    else:
        m["f1_score"] = float(f1_score(labels, preds, average="weighted", zero_division=0))
    return m


class EarlyStopping:
    """utils/early_stopping.py:4-56: stop after `patience` epochs without a val-loss decrease of
    more than `delta`; checkpoint on every improvement."""

    def __init__(self, patience=7, delta=0.0, path="checkpoint.pt", logger=None):
        self.patience, self.delta, self.path, self.logger = patience, delta, path, logger
        self.counter, self.best_score, self.early_stop = 0, None, False

    def __call__(self, val_loss, save_fn):
        score = -val_loss
        if self.best_score is None or score >= self.best_score + self.delta:
            self.best_score = score
            save_fn(self.path)
            self.counter = 0
        else:
            self.counter += 1
            if self.counter >= self.patience:
                self.early_stop = True


# ------------------------------------------------------------------------- families
class Family:
    """What differs between the four folders: factory, sampler, decode span, GPU transform."""

    def __init__(self, name, prefix, model_dir, batch_size, epochs, lr, wd, optimizer):
        self.name, self.prefix, self.model_dir = name, prefix, model_dir
        self.batch_size, self.epochs, self.lr, self.wd, self.optimizer = batch_size, epochs, lr, wd, optimizer

    def load_clip(self, src, sampler, path, num_frames):
        """Decoded uint8 frames the transform consumes: the sampled frames (ViViT/TimeSformer,
        resized to 224 as dataset.py:271-277), or every frame of the sampled span (Swin/ResNet3D
        `get_clip(idx0/fps, (idxN+1)/fps)`, then UniformTemporalSubsample on the GPU)."""
        idx = sampler.get_sampling_indices(str(path), src.total_frames)
        if isinstance(idx, tuple):
            idx = idx[0]
        if self.name in ("vivit", "timesformer"):
            fr = src.read(idx)  # resized to 224x224 on the GPU (to_model_input), as dataset.py:271-277
            if len(fr) < num_frames:  # pad by repeating the last frame (dataset.py:256-265)
                fr = np.concatenate([fr, np.repeat(fr[-1:], num_frames - len(fr), 0)])
            return fr[:num_frames]
        lo, hi = int(min(idx)), int(max(idx))
        return src.read(list(range(lo, hi + 1)))

    def to_model_input(self, frames_u8: torch.Tensor, num_frames, div255=False, train=False):
        """train: the Swin / ResNet3D train chain (RandomShortSideScale, RandomCrop, RandomHorizontalFlip;
        dataset.py:151-163 / :176-182) instead of the eval chain; ViViT / TimeSformer have one chain."""
        from . import preprocess as pp
        if self.name in ("vivit", "timesformer") and tuple(frames_u8.shape[-3:-1]) != (224, 224):
            frames_u8 = pp.cv2_resize_u8(frames_u8, (224, 224))  # cv2.resize INTER_LINEAR (dataset.py:271-277)
        if self.name == "vivit":
            return pp.vivit_preprocess(frames_u8)
        if self.name == "timesformer":
            return pp.timesformer_preprocess(frames_u8)
        if train:
            return pp.video_train_transform(frames_u8, num_frames, div255=div255)[0]
        return pp.video_eval_transform(frames_u8, num_frames, div255=div255)

    def create_model(self, args, class_labels, device, logger):
        if self.name == "vivit":
            from .vivit import create_model
            return create_model(args.model_name, args.num_classes, class_labels, args.num_frames, device, logger)
        if self.name == "timesformer":
            from .timesformer import create_model
            return create_model(args.model_name, args.num_classes, class_labels, args.num_frames, device, logger)
        if self.name == "swin":
            from .swin3d import create_model
            return create_model(logger, args.model_size, getattr(args, "pretrained", True), args.num_classes, device=device)
        from .resnet3d import create_model
        return create_model(logger, device=device)

    def logits(self, model, x):
        if self.name in ("vivit", "timesformer"):
            return model(pixel_values=x).logits
        return model(x)


FAMILIES = {
    "vivit": Family("vivit", "vivit-classifier", "vivit-models", 4, 40, 1e-3, 0.01, "adamw"),
    "timesformer": Family("timesformer", "timesformer-classifier", "timesformer-models", 4, 40, 1e-3, 0.01, "adamw"),
    "swin": Family("swin", "swin3d-classifier", "swin-models", 8, 30, 1e-4, 0.05, "adamw"),
    "resnet3d": Family("resnet3d", "resnet3d-classifier", "resnet3d-models", 8, 30, 1e-3, 0.0, "adam"),
}


def build_parser(fam: Family, inference: bool):
    p = argparse.ArgumentParser(description=f"{fam.name} video classifier (libvclip, MI355X)")
    if inference:
        p.add_argument("--video_path", type=str, required=True)
        p.add_argument("--model_path", type=str, required=True)
        p.add_argument("--log_dir", type=str, default="logs")
        p.add_argument("--num_frames", type=int, default=32)
        p.add_argument("--sampling_method", type=str, default="uniform", choices=SAMPLING)
        if fam.name != "resnet3d":
            p.add_argument("--num_classes", type=int, default=2)
        if fam.name == "swin":
            p.add_argument("--model_size", type=str, default="tiny", choices=["tiny", "small", "base", "base_in22k"])
        if fam.name in ("vivit", "timesformer"):
            p.add_argument("--save_viz", action="store_true")
        else:
            p.add_argument("--visualize", action="store_true")
        return p
    required = fam.name in ("swin", "resnet3d")
    p.add_argument("--data_dir", type=str, required=True)
    p.add_argument("--test_data_dir", type=str, default=None)
    p.add_argument("--log_dir", type=str, default=None if required else "logs", required=required)
    p.add_argument("--model_dir", type=str, default=None if required else fam.model_dir, required=required)
    for s in ("train", "val", "test"):
        p.add_argument(f"--{s}_sampling", type=str, default="uniform", choices=SAMPLING)
    p.add_argument("--num_frames", type=int, default=32)
    if fam.name == "vivit":
        p.add_argument("--model_name", type=str, default="google/vivit-b-16x2-kinetics400")
    elif fam.name == "timesformer":
        p.add_argument("--model_name", type=str, default="facebook/timesformer-base-finetuned-k400")
    elif fam.name == "swin":
        p.add_argument("--model_size", type=str, default="tiny", choices=["tiny", "small", "base", "base_in22k"])
        p.add_argument("--pretrained", action="store_true")
    if fam.name != "resnet3d":
        p.add_argument("--num_classes", type=int, default=2)
    p.add_argument("--batch_size", type=int, default=fam.batch_size)
    p.add_argument("--num_workers", type=int, default=4)
    p.add_argument("--epochs", type=int, default=fam.epochs)
    p.add_argument("--learning_rate", type=float, default=fam.lr)
    if fam.name != "resnet3d":
        p.add_argument("--weight_decay", type=float, default=fam.wd)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--patience", type=int, default=7)
    p.add_argument("--early_stopping_delta", type=float, default=0.001)
    # resnet50-3d-video/main.py:53-58, offered by every family here (evaluate a checkpoint, no training)
    p.add_argument("--skip_train", action="store_true")
    p.add_argument("--checkpoint_path", type=str, default=None)
    if fam.name == "resnet3d":
        p.add_argument("--weighted_sampling", action="store_true")
    return p


def _device():
    import os
    if not torch.cuda.is_available():
        raise RuntimeError("vclip_amd runs on the GPU only (MI355X); no CPU execution path")
    return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))


def _loaders(fam, args, logger, exp_dir):
    """({split: loader}, class labels) from the folder's own data_config drop-in, so `--num_workers`
    decode workers run as in the reference (vivit_transformer/main.py:93, videoswintransformer/
    main.py:105, resnet50-3d-video/main.py:94-97 with the sampled-index CSVs in the experiment dir).
    `--skip_train` builds the test split only (resnet50-3d-video/main.py:53-58 evaluates a checkpoint)."""
    from torch.utils.data import DataLoader

    from .data_config import FOLDERS, DeviceClipLoader, swin
    mod = FOLDERS[fam.name]
    methods = {s: getattr(args, f"{s}_sampling") for s in ("train", "val", "test")}
    hf = fam.name in ("vivit", "timesformer")
    binary = ["non-referral", "referral"]  # Swin3D / ResNet3D label = (folder == 'referral')
    if not args.skip_train:
        if hf:
            return mod.create_dataloaders(args, methods, logger)
        if fam.name == "swin":
            return mod.create_dataloaders(args, logger), binary
        return mod.create_dataloaders(args, logger, log_dir=str(exp_dir))[1], binary
    if fam.name == "resnet3d":
        # resnet50-3d-video/main.py:94-98 builds every split with the experiment dir before it looks
        # at --skip_train, so the sampled-index CSVs (its only golden artefact) are written for train,
        # val and test; a dataset without train/val splits still gets its test CSV
        try:
            return {"test": mod.create_dataloaders(args, logger, log_dir=str(exp_dir))[1]["test"]}, binary
        except Exception as e:  # noqa: BLE001 - the reference raises here; evaluating the test split is still possible
            logger.warning(f"create_dataloaders failed ({e}); building the test split only")
            ds = mod.VideoDataset(args.test_data_dir or args.data_dir, mode="test", sampling_method=methods["test"],
                                  num_frames=args.num_frames, logger=logger, log_dir=str(exp_dir))
            ds.save_sampled_indices()
            return {"test": DeviceClipLoader(ds, batch_size=args.batch_size, num_workers=args.num_workers,
                                             collate_fn=swin.video_collate_fn)}, binary
    root = args.test_data_dir or args.data_dir
    ds = mod.VideoDataset(root, mode="test", sampling_method=methods["test"], num_frames=args.num_frames,
                          logger=logger)
    if hf:
        loader = DataLoader(ds, batch_size=args.batch_size, shuffle=False, num_workers=args.num_workers,
                            collate_fn=mod.video_collate_fn)
        return {"test": loader}, ds.class_labels
    return {"test": DeviceClipLoader(ds, batch_size=args.batch_size, num_workers=args.num_workers,
                                     collate_fn=swin.video_collate_fn)}, binary


def _batches(fam, loader, args, device):
    """(model input, labels) on the device per loader batch: the HF folders' uint8 clips through the
    GPU processor (trainer.py:62-104), the Swin3D / ResNet3D clips [B, n, C, T, H, W] flattened to
    [B * n, C, T, H, W] (videoswintransformer/.../trainers/trainer.py:105-111)."""
    for batch in loader:
        if isinstance(batch, dict):
            pv = batch["pixel_values"]
            fr = torch.from_numpy(np.stack(pv)) if isinstance(pv, (list, tuple)) else torch.as_tensor(pv)
            x = fam.to_model_input(fr.to(device), args.num_frames)
            yield x, batch["labels"].reshape(-1).to(device)
        else:
            clips, labels = batch
            yield clips.reshape(-1, *clips.shape[2:]).to(device), labels.reshape(-1).to(device)


def _load_weights(model, path, logger, fam):
    from .checkpoint import load_reference_checkpoint
    ck, sd = load_reference_checkpoint(path, vivit_keys=fam.name == "vivit")
    model.load_state_dict(sd)
    logger.info(f"Loaded weights from {path}")
    return ck


@torch.no_grad()
def evaluate(fam, model, loader, args, device, class_names, exp_dir, method, logger):
    model.eval()
    probs, preds, labels = [], [], []
    for x, y in _batches(fam, loader, args, device):
        try:
            p = torch.softmax(fam.logits(model, x).float(), dim=1)
        except Exception as e:  # noqa: BLE001 - evaluator.py: log and skip the batch
            logger.error(f"Error in test batch: {str(e)}")
            continue
        probs.append(p.cpu().numpy())
        preds += p.argmax(1).tolist()
        labels += y.tolist()
    probs = np.concatenate(probs) if probs else np.zeros((0, len(class_names)))
    m = compute_metrics(labels, preds, probs, class_names)
    with open(Path(exp_dir) / f"test_metrics_{method}.json", "w") as f:
        json.dump(m, f, indent=4)
    logger.info(f"Test accuracy {m['accuracy']:.4f}  F1 {m.get('f1_score', 0):.4f}  AUROC {m.get('auroc', 0):.4f}")
    return m


def run_main(fam_name, argv=None):
    fam = FAMILIES[fam_name]
    args = build_parser(fam, inference=False).parse_args(argv)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    random.seed(args.seed)
    exp = ExperimentLogger(args.log_dir, prefix=fam.prefix)
    logger = exp.get_logger()
    logger.info(f"Arguments: {vars(args)}")
    device = _device()
    loaders, class_labels = _loaders(fam, args, logger, exp.get_experiment_dir())
    if not hasattr(args, "num_classes"):
        args.num_classes = len(class_labels)
    model = fam.create_model(args, class_labels, device, logger)
    if args.checkpoint_path:
        _load_weights(model, args.checkpoint_path, logger, fam)
    history = {"train_loss": [], "train_acc": [], "val_loss": [], "val_acc": []}
    if not args.skip_train:
        from .optim import AdamW
        # ResNet3D: torch.optim.Adam(model.parameters(), lr) (resnet50-3d-video/main.py:153) = AdamW with
        # weight decay 0; its BatchNorm running statistics carry no gradient and are skipped
        opt = AdamW([q for q in model.parameters() if q.requires_grad], lr=args.learning_rate,
                    weight_decay=getattr(args, "weight_decay", 0.0))
        crit = torch.nn.CrossEntropyLoss()
        model_dir = Path(args.model_dir)
        model_dir.mkdir(parents=True, exist_ok=True)
        best_path = model_dir / f"best_model_{args.train_sampling}.pth"
        stopper = EarlyStopping(args.patience, args.early_stopping_delta, exp.get_experiment_dir() / "checkpoint.pt")
        best_val = float("inf")
        for epoch in range(args.epochs):
            model.train()
            tl, tc, tn = 0.0, 0, 0
            for x, y in _batches(fam, loaders["train"], args, device):
                try:  # trainer.py:133-167: a failing batch is logged and skipped
                    opt.zero_grad()
                    logits = fam.logits(model, x)
                    loss = crit(logits, y)
                    loss.backward()
                    opt.step()
                    tl += loss.item() * len(y)
                    tc += int((logits.argmax(1) == y).sum())
                    tn += len(y)
                except Exception as e:  # noqa: BLE001
                    logger.error(f"Error in training batch: {str(e)}")
                    continue
            model.eval()
            vl, vc, vn = 0.0, 0, 0
            with torch.no_grad():
                for x, y in _batches(fam, loaders["val"], args, device):
                    try:  # trainer.py:192-210
                        logits = fam.logits(model, x)
                        vl += float(crit(logits, y)) * len(y)
                        vc += int((logits.argmax(1) == y).sum())
                        vn += len(y)
                    except Exception as e:  # noqa: BLE001
                        logger.error(f"Error in validation batch: {str(e)}")
                        continue
            # a batch that fails is logged and skipped (trainer.py:165-167), but an epoch in which EVERY
            # batch failed (e.g. a kernel fault on each launch) must not go on to save a "best" model
            if tn == 0 and len(loaders["train"]) > 0:
                raise RuntimeError(f"epoch {epoch + 1}: every training batch failed (see the log)")
            if vn == 0 and len(loaders["val"]) > 0:
                raise RuntimeError(f"epoch {epoch + 1}: every validation batch failed (see the log)")
            tr_loss, tr_acc = tl / max(tn, 1), tc / max(tn, 1)
            va_loss, va_acc = vl / max(vn, 1), vc / max(vn, 1)
            for k, v in (("train_loss", tr_loss), ("train_acc", tr_acc), ("val_loss", va_loss), ("val_acc", va_acc)):
                history[k].append(v)
            logger.info(f"Epoch {epoch + 1}/{args.epochs}: train loss {tr_loss:.4f} acc {tr_acc:.4f} | "
                        f"val loss {va_loss:.4f} acc {va_acc:.4f}")

            def save(path, epoch=epoch, va_loss=va_loss, va_acc=va_acc):
                ck = {"epoch": epoch, "model_state_dict": model.state_dict(), "optimizer_state_dict": opt.state_dict(),
                      "val_loss": va_loss, "val_acc": va_acc, "history": history}
                if hasattr(model, "config"):  # HF families: vivit trainer.py:291-305 (and TimeSformer's)
                    ck.update({"config": model.config.to_dict(), "id2label": model.config.id2label,
                               "label2id": model.config.label2id, "num_frames": args.num_frames,
                               "train_sampling": args.train_sampling, "val_sampling": args.val_sampling,
                               "test_sampling": args.test_sampling})
                # (Swin3D: videoswintransformer/.../trainers/trainer.py:191-198 saves the six keys above)
                torch.save(ck, path)

            if va_loss < best_val:  # trainer.py:231-236 + _save_best_model
                best_val = va_loss
                save(best_path)
                logger.info(f"Saved best model to {best_path}")
            stopper(va_loss, save)
            if stopper.early_stop:
                logger.info("Early stopping triggered")
                break
        _load_weights(model, best_path, logger, fam)
    m = evaluate(fam, model, loaders["test"], args, device, class_labels, exp.get_experiment_dir(),
                 args.test_sampling, logger)
    logger.info("Training and evaluation pipeline completed successfully")
    return m, history, exp.get_experiment_dir()


def run_inference(fam_name, argv=None):
    fam = FAMILIES[fam_name]
    args = build_parser(fam, inference=True).parse_args(argv)
    exp = ExperimentLogger(args.log_dir, prefix=f"{fam.prefix}-inference")
    logger = exp.get_logger()
    device = _device()
    from .checkpoint import load_reference_checkpoint
    ck, sd = load_reference_checkpoint(args.model_path, vivit_keys=fam.name == "vivit")
    id2label = {int(k): v for k, v in (ck.get("id2label") or {0: "non-referral", 1: "referral"}).items()}
    class_labels = [id2label[i] for i in sorted(id2label)]
    args.num_classes = len(class_labels)
    if fam.name in ("vivit", "timesformer"):
        args.model_name = "checkpoint"
        if ck.get("config"):
            cfg = dict(ck["config"])
            if fam.name == "vivit":
                from .vivit import VivitConfig, VivitForVideoClassification
                model = VivitForVideoClassification(VivitConfig.from_dict(cfg)).to(device).eval()
            else:
                from .timesformer import TimesformerConfig, TimesformerForVideoClassification
                model = TimesformerForVideoClassification(TimesformerConfig.from_dict(cfg)).to(device).eval()
        else:
            model = fam.create_model(args, class_labels, device, logger)
    else:
        model = fam.create_model(args, class_labels, device, logger)
    model.load_state_dict(sd)
    model.eval()  # the reference inference scripts' model.eval()
    src = video_io.open_video(args.video_path)
    if fam.name in ("vivit", "timesformer"):
        sampler = sampling.VivitSampler(args.num_frames, args.sampling_method, logger)
    elif fam.name == "swin":
        sampler = _SwinInferenceSampler(args.num_frames, args.sampling_method, logger, src.fps)
    else:
        sampler = sampling.Resnet3dInferenceSampler(args.num_frames, args.sampling_method, logger,
                                                    fps_of=lambda p: src.fps)
    frames = torch.from_numpy(fam.load_clip(src, sampler, args.video_path, args.num_frames)).to(device)
    # the Swin / ResNet3D inference scripts divide by 255 before Normalize (resnet50-3d-video/inference.py:382-394)
    x = fam.to_model_input(frames.unsqueeze(0), args.num_frames, div255=True)
    t0 = time.perf_counter()
    with torch.no_grad():
        probs = torch.softmax(fam.logits(model, x).float(), dim=1)
    torch.cuda.synchronize()
    pred = int(probs.argmax(1))
    conf = float(probs[0, pred])
    name = id2label[pred]
    logger.info(f"Prediction: {name}  Confidence: {conf:.4f}  ({(time.perf_counter() - t0) * 1e3:.1f} ms)")
    print(f"Predicted class: {name}")
    print(f"Confidence: {conf:.4f}")
    res = {"video_path": str(args.video_path), "predicted_class": name,
           "class_id": id2label.get(name, -1),  # (sic) the reference looks the name up in id2label: -1
           "confidence": conf, "class_mapping": {str(k): v for k, v in id2label.items()}}
    out = exp.get_experiment_dir() / "inference_results"
    out.mkdir(parents=True, exist_ok=True)
    with open(out / f"{Path(args.video_path).stem}_result.json", "w") as f:
        json.dump(res, f, indent=4)
    return res


class _SwinInferenceSampler:
    """videoswintransformer/inference.py:94-185 (module function, reseeds 42 per call)."""

    def __init__(self, num_frames, method, logger, fps):
        self.num_frames, self.method, self.logger, self.fps = num_frames, method, logger, fps

    def get_sampling_indices(self, video_path, total_frames):
        return sampling.swin_inference_sampling_indices(video_path, total_frames, self.num_frames, self.method,
                                                        self.logger, fps_of=lambda p: self.fps)

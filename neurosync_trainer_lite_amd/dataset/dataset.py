"""Drop-in for dataset/dataset.py (AudioFacialDataset, dataloaders).

Same windows in the same order as the reference's ``process_example``
(dataset.py:58-98): stride-1 windows of ``micro_batch_size`` frames, plus one
tail window when the clip length is not a multiple of it (tail shorter than a
window is completed by its mirror image).  Windows are NOT materialised up
front (the reference keeps ~162 KB per window in host RAM, README.md:34):
each clip is stored once as float32 and a window is sliced when requested.
Values are identical: the reference casts each window float64 -> float32
elementwise, here the clip is cast once.

Batches are fetched whole (``__getitems__``, which torch's DataLoader and
random_split's Subset call with a batch's indices): the windows are copied
straight into one page-locked (pinned) host batch from the caching host
allocator, so ``src.to(device, non_blocking=True)`` in the training loop is an
asynchronous DMA, and the allocator keeps a pinned block out of reuse until the
copies that read it have finished.
"""
import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, random_split

from .data_processing import load_data


def prepare_dataloader_with_split(config, val_split=0.1):
    """dataset.py:12-21."""
    dataset = AudioFacialDataset(config)
    val_size = int(len(dataset) * val_split)
    train_size = len(dataset) - val_size
    train_dataset, val_dataset = random_split(dataset, [train_size, val_size])
    train_dataloader = DataLoader(train_dataset, batch_size=config['batch_size'], shuffle=True,
                                  collate_fn=AudioFacialDataset.collate_fn)
    val_dataloader = DataLoader(val_dataset, batch_size=config['batch_size'], shuffle=False,
                                collate_fn=AudioFacialDataset.collate_fn)
    return train_dataset, val_dataset, train_dataloader, val_dataloader


def prepare_dataloader(config):
    """dataset.py:23-26."""
    dataset = AudioFacialDataset(config)
    dataloader = DataLoader(dataset, batch_size=config['batch_size'], shuffle=True,
                            collate_fn=AudioFacialDataset.collate_fn)
    return dataset, dataloader


def _rows(n, start, end):
    """Length of x[start:end] for len(x) == n (Python slice semantics)."""
    return len(range(n)[start:end])


def window_plan(n_audio, n_facial, window):
    """[(start, is_tail)] for one clip; raises ValueError exactly where the
    reference's process_example would fail on a shape mismatch."""
    max_frames = max(n_audio, n_facial)
    plan = []
    for start in range(0, max_frames - window + 1):
        for n in (n_audio, n_facial):
            want = len(range(window)[:min(window, n - start)])
            if want != _rows(n, start, start + window):
                raise ValueError("could not broadcast window at %d (clip length %d)" % (start, n))
        plan.append((start, False))
    if max_frames % window != 0:
        start = max_frames - window
        for n in (n_audio, n_facial):
            got = _rows(n, start, max_frames)
            if window - got > got:
                raise ValueError("could not broadcast tail window (clip length %d < %d)" % (n, window))
        plan.append((start, True))
    return plan


def _window(x, start, window, tail, end):
    seg = np.zeros((window, x.shape[1]), dtype=np.float32)
    part = x[start:start + window] if not tail else x[start:end]
    seg[:len(part)] = part
    if tail and len(part) < window:
        seg[len(part):] = part[::-1][:window - len(part)]
    return seg


class AudioFacialDataset(Dataset):
    def __init__(self, config):
        self.root_dir = config['root_dir']
        self.sr = config['sr']
        self.frame_rate = config['frame_rate']
        self.micro_batch_size = config['micro_batch_size']
        self.processed_folders = set()
        self.clips = []   # [(audio f32 [N, 256], facial f32 [N, 61])]
        self.index = []   # [(clip, start, is_tail)]
        self.pin = torch.cuda.is_available()
        for audio_features, facial_data in load_data(self.root_dir, self.sr, self.processed_folders,
                                                     include_fast=config.get('include_fast', True),
                                                     include_slow=config.get('include_slow', False)):
            self.add_clip(audio_features, facial_data)

    def add_clip(self, audio_features, facial_data):
        plan = window_plan(len(audio_features), len(facial_data), self.micro_batch_size)
        c = len(self.clips)
        self.clips.append((np.ascontiguousarray(audio_features, dtype=np.float32),
                           np.ascontiguousarray(facial_data, dtype=np.float32)))
        self.index.extend((c, s, t) for s, t in plan)

    @property
    def examples(self):
        return _LazyExamples(self)

    def __len__(self):
        return len(self.index)

    def __getitem__(self, idx):
        c, start, tail = self.index[idx]
        audio, facial = self.clips[c]
        end = max(len(audio), len(facial))
        w = self.micro_batch_size
        return (torch.from_numpy(_window(audio, start, w, tail, end)),
                torch.from_numpy(_window(facial, start, w, tail, end)))

    def __getitems__(self, indices):
        """A whole batch (torch DataLoader batched fetch): windows copied into one
        pinned (src, trg) pair, in index order."""
        w = self.micro_batch_size
        a0, f0 = self.clips[self.index[indices[0]][0]] if len(indices) else (np.zeros((0, 256)), np.zeros((0, 61)))
        src = torch.empty((len(indices), w, a0.shape[1]), dtype=torch.float32, pin_memory=self.pin)
        trg = torch.empty((len(indices), w, f0.shape[1]), dtype=torch.float32, pin_memory=self.pin)
        s_np, t_np = src.numpy(), trg.numpy()
        for i, idx in enumerate(indices):
            c, start, tail = self.index[idx]
            audio, facial = self.clips[c]
            end = max(len(audio), len(facial))
            for x, out in ((audio, s_np[i]), (facial, t_np[i])):
                if not tail and start + w <= len(x):
                    out[:] = x[start:start + w]  # the common case: one contiguous copy
                else:
                    out[:] = _window(x, start, w, tail, end)
        return _Batch(src, trg)

    @staticmethod
    def collate_fn(batch):
        """dataset.py:51-56 (every window has the same length: a stack); a batch
        fetched whole by __getitems__ passes through."""
        if isinstance(batch, _Batch):
            return batch.src, batch.trg
        src_batch, trg_batch = zip(*batch)
        return torch.stack(src_batch), torch.stack(trg_batch)

    def process_example(self, audio_features, facial_data):
        """dataset.py:58-98, materialised (API compatibility)."""
        w = self.micro_batch_size
        end = max(len(audio_features), len(facial_data))
        return [(torch.from_numpy(_window(np.asarray(audio_features, dtype=np.float32), s, w, t, end)),
                 torch.from_numpy(_window(np.asarray(facial_data, dtype=np.float32), s, w, t, end)))
                for s, t in window_plan(len(audio_features), len(facial_data), w)]


class _Batch(list):
    """(src [B, T, 256], trg [B, T, 61]) as fetched by __getitems__.  It is also
    the list of per-window (src_i, trg_i) pairs (views of the pinned batch), so a
    DataLoader with torch's default_collate (or any collate that takes a list of
    samples) still works; AudioFacialDataset.collate_fn takes the pinned tensors
    whole."""

    def __init__(self, src, trg):
        super().__init__(zip(src.unbind(0), trg.unbind(0)))
        self.src, self.trg = src, trg


class _LazyExamples:
    """Sequence view standing in for the reference's ``examples`` list."""

    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self.ds[j] for j in range(*i.indices(len(self.ds)))]
        return self.ds[i]

    def __iter__(self):
        return (self.ds[i] for i in range(len(self.ds)))

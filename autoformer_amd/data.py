"""Training data path: the reference's VCTK utterance loader (util/data_loader.py) with the same
on-disk format and sampling, plus an MI355X feed that keeps the next batch's H2D copy off the
training stream.

On-disk format (util/data_loader.py:29-31, make_metadata.ipynb): ``<root>/train.pkl`` holds a
list with one entry per speaker, ``[speaker_id, emb (256,) float32, 'spk/utt1.npy', ...]``;
every ``.npy`` is a log-mel spectrogram ``(T_utt, 80)`` float32.

* ``Utterances(root_dir, len_crop)`` / ``get_loader(...)`` keep the reference constructor, the
  dataset item ``(uttr (len_crop, 80), emb (256,))`` and the DataLoader settings
  (shuffle, drop_last, per-worker numpy seeding; data_loader.py:88-102).  Item sampling draws
  from ``np.random`` in the reference's order -- utterance index, then crop offset only when the
  utterance is longer than ``len_crop`` (data_loader.py:63-81) -- so a seeded run picks the
  same crops.  The mels are read by a thread pool (``np.load`` releases the GIL on file IO)
  instead of one ``multiprocessing.Process`` per ten speakers through a ``Manager`` list.
* ``DeviceFeed(loader, device)`` turns any ``(uttr, emb)`` batch iterator into device tensors:
  a background thread collates each batch into a reused pinned host buffer and copies it with
  ``non_blocking`` on a dedicated copy stream, two batches ahead; the consumer's stream waits on
  an event only when it takes the batch (2.6 MB of H2D per B=64/T=128 batch).
"""
from __future__ import annotations

import os
import pickle
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from torch.utils import data


def _load_speaker(root_dir, entry):
    out = list(entry[:2])
    for rel in entry[2:]:
        out.append(np.load(os.path.join(root_dir, rel.replace("\\", "/"))))
    return out


class Utterances(data.Dataset):
    """Dataset of speakers; item = one random utterance of speaker `index`, randomly cropped
    or zero-padded (at the end) to `len_crop` frames, with the speaker embedding."""

    def __init__(self, root_dir, len_crop, num_threads=None):
        self.root_dir = root_dir
        self.len_crop = len_crop
        with open(os.path.join(root_dir, "train.pkl"), "rb") as f:
            meta = pickle.load(f)  # the dataset's own metadata file (data_loader.py:29-31)
        threads = num_threads or min(32, (os.cpu_count() or 4))
        with ThreadPoolExecutor(max_workers=threads) as pool:
            self.train_dataset = list(pool.map(lambda e: _load_speaker(root_dir, e), meta))
        self.num_tokens = len(self.train_dataset)

    def crop(self, mel, rng=np.random):
        """data_loader.py:69-79: pad short utterances with zeros at the end, crop long ones at a
        uniform offset in [0, T - len_crop) (one rng draw, only when T > len_crop)."""
        T = mel.shape[0]
        if T < self.len_crop:
            out = np.zeros((self.len_crop, mel.shape[1]), dtype=mel.dtype)
            out[:T] = mel
            return out
        if T > self.len_crop:
            left = rng.randint(T - self.len_crop)
            return mel[left:left + self.len_crop, :]
        return mel

    def __getitem__(self, index):
        spk = self.train_dataset[index]
        u = np.random.randint(2, len(spk))  # which utterance (data_loader.py:68)
        return self.crop(spk[u]), spk[1]

    def __len__(self):
        return self.num_tokens


def get_loader(root_dir, dim_neck=44, batch_size=2, len_crop=176, num_workers=0):
    """util/data_loader.py:88-102: shuffled, drop_last DataLoader over Utterances."""
    dataset = Utterances(root_dir, len_crop)

    def worker_init_fn(_):
        np.random.seed(torch.initial_seed() % (2 ** dim_neck))

    return data.DataLoader(dataset=dataset, batch_size=batch_size, shuffle=True, num_workers=num_workers,
                           drop_last=True, worker_init_fn=worker_init_fn)


class DeviceFeed:
    """Iterate device batches (x_real (B, T, 80), emb (B, E)) from a host batch iterator.

    A background thread pulls host batches, copies them into pinned buffers and issues the
    H2D copies on a dedicated copy stream, `depth` batches ahead; the consumer only makes its
    current stream wait on the batch's event.  The training thread therefore pays neither the
    collation nor the copy (measured, tools/feed_bench.py)."""

    def __init__(self, loader, device, depth=2, repeat=False):
        if not torch.cuda.is_available():
            raise RuntimeError("DeviceFeed needs the HIP device (no CPU fallback)")
        self.loader = loader
        self.device = torch.device(device)
        self.depth = depth
        self.repeat = repeat  # cycle over epochs in one producer (the reference's train loop
                              # re-creates its iterator when an epoch ends, train.py:69-73)
        self.copy = torch.cuda.Stream(device=self.device)

    def _produce(self, q, stop):
        pinned = {}

        def pin(key, t):
            t = torch.as_tensor(t)
            buf = pinned.get(key)
            if buf is None or buf.shape != t.shape:
                buf = torch.empty(t.shape, dtype=torch.float32, pin_memory=True)
                pinned[key] = buf
            buf.copy_(t)
            return buf

        try:
            torch.cuda.set_device(self.device)
            while not stop.is_set():
                for uttr, emb in self.loader:
                    if stop.is_set():
                        break
                    hx, he = pin("x", uttr), pin("e", emb)
                    with torch.cuda.stream(self.copy):
                        x = hx.to(self.device, non_blocking=True)
                        e = he.to(self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.copy)
                    ev.synchronize()  # this thread only: the pinned buffers may be refilled after it
                    q.put((x, e, ev))
                if not self.repeat:
                    break
        except BaseException as exc:  # surface loader errors in the consumer
            q.put(exc)
            return
        q.put(None)

    def __iter__(self):
        import queue
        import threading

        q = queue.Queue(maxsize=self.depth)
        stop = threading.Event()
        th = threading.Thread(target=self._produce, args=(q, stop), daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                x, e, ev = item
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                x.record_stream(cur)
                e.record_stream(cur)
                yield x, e
        finally:
            stop.set()
            while th.is_alive():  # drain so the producer can finish its last put
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(0.01)

    def __len__(self):
        return len(self.loader)

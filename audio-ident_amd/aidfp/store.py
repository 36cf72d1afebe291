"""Persistence of the fingerprint index: the OLAF_DB directory.

The reference keeps Olaf's LMDB environment in `settings.olaf_lmdb_path`
(audio-ident-service/app/settings.py:39), created by `_get_olaf_env`
(app/audio/fingerprint.py:71-84); every `olaf_c store` / `del` is one LMDB write
transaction (fingerprint.py:117-140, :239-262). Here the index lives on the GPU and
the directory holds a snapshot plus a write-ahead journal:

  tracks.json          manifest and commit point: {"version", "snapshot", "journal",
                       "ids": {name: track id}, "next"} as of the snapshot
  index.<g>.aidfp      snapshot of generation g (aid_index_save: AIDFPIX1 file)
  journal.<g>.aidfj    operations since that snapshot, appended and fsynced one per
                       store/delete: O(size of the track) bytes per call

A store appends the track's records (8 B each) to the journal; a delete appends a
tombstone. When the journal outgrows the snapshot (and a floor, default 64 MiB) the
store checkpoints: removed tracks' postings are compacted away on the device
(aid_index_compact), a new snapshot and an empty journal of generation g+1 are
written, and the manifest is replaced atomically (os.replace). A crash at any point
leaves either the old or the new generation complete; a torn journal tail (a crash
inside an append) is detected by its CRC and cut off at load.

Ingest of N tracks therefore writes O(total postings) bytes, not O(N^2): every
posting is written once to the journal and, amortised, a bounded number of times
into snapshots (each checkpoint at least doubles the journal bytes it folds in).
"""

from __future__ import annotations

import json
import logging
import os
import struct
import zlib
from pathlib import Path

import numpy as np

logger = logging.getLogger(__name__)

MANIFEST = "tracks.json"
LEGACY_SNAPSHOT = "index.aidfp"  # round-1 layout: snapshot only, no journal
JOURNAL_MAGIC = b"AIDJ"
OP_STORE, OP_DELETE = 1, 2
_HDR = struct.Struct("<4sIIIQ")  # magic, op, track id, name bytes, record count
_CRC = struct.Struct("<I")


class StoreCorrupt(Exception):
    """The snapshot or manifest cannot be read (the journal tail is repaired instead)."""


def _fsync_dir(d: Path) -> None:
    try:
        fd = os.open(d, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


def encode_entry(op: int, track: int, name: str, recs: np.ndarray | None = None) -> bytes:
    nb = name.encode("utf-8")
    body = np.ascontiguousarray(recs, dtype="<u8").tobytes() if recs is not None else b""
    head = _HDR.pack(JOURNAL_MAGIC, op, int(track), len(nb), len(body) // 8)
    crc = zlib.crc32(body, zlib.crc32(nb, zlib.crc32(head)))
    return head + nb + body + _CRC.pack(crc)


def read_journal(path: Path) -> tuple[list[tuple[int, int, str, np.ndarray | None]], int]:
    """Parse a journal; returns (entries, bytes of the valid prefix). Parsing stops at the first
    incomplete or corrupt entry (a torn append)."""
    if not path.exists():
        return [], 0
    data = path.read_bytes()
    out, pos = [], 0
    while pos + _HDR.size <= len(data):
        magic, op, track, nlen, n = _HDR.unpack_from(data, pos)
        end = pos + _HDR.size + nlen + 8 * n + _CRC.size
        if magic != JOURNAL_MAGIC or op not in (OP_STORE, OP_DELETE) or end > len(data):
            break
        nb = data[pos + _HDR.size: pos + _HDR.size + nlen]
        body = data[pos + _HDR.size + nlen: end - _CRC.size]
        crc = zlib.crc32(body, zlib.crc32(nb, zlib.crc32(data[pos: pos + _HDR.size])))
        if crc != _CRC.unpack_from(data, end - _CRC.size)[0]:
            break
        try:
            name = nb.decode("utf-8")
        except UnicodeDecodeError:
            break
        recs = np.frombuffer(body, dtype="<u8").astype(np.uint64) if op == OP_STORE else None
        out.append((op, track, name, recs))
        pos = end
    return out, pos


class IndexStore:
    """Snapshot + journal persistence of one engine's index (see the module docstring)."""

    def __init__(self, db_dir: Path, checkpoint_min_bytes: int = 64 << 20):
        self.db_dir = Path(db_dir)
        self.checkpoint_min_bytes = int(checkpoint_min_bytes)
        self.snapshot: str | None = None
        self.journal = "journal.0.aidfj"
        self.gen = 0
        self.journal_bytes = 0
        self.snapshot_bytes = 0
        self.loaded = False

    # -- load --
    def load(self, engine) -> tuple[dict[str, int], int, list]:
        """Load the snapshot into `engine`; returns (ids, next id) as of the snapshot and the
        journal's entries (op, track, name, records) for the caller to replay in order.
        Raises StoreCorrupt / the engine's error if the snapshot cannot be loaded; the engine
        must then be discarded."""
        man = self.db_dir / MANIFEST
        ids: dict[str, int] = {}
        nxt = 0
        if man.exists():
            try:
                d = json.loads(man.read_text())
                ids = {str(k): int(v) for k, v in d["ids"].items()}
                nxt = int(d["next"])
            except (ValueError, KeyError, TypeError, AttributeError) as exc:
                raise StoreCorrupt(f"unreadable index manifest {man}: {exc}") from exc
            self.snapshot = d.get("snapshot", LEGACY_SNAPSHOT)
            self.journal = d.get("journal", "journal.legacy.aidfj")
            self.gen = int(d.get("gen", 0))
        elif (self.db_dir / LEGACY_SNAPSHOT).exists():
            raise StoreCorrupt(f"{self.db_dir / LEGACY_SNAPSHOT} exists without its manifest {MANIFEST}")
        if self.snapshot is not None:
            snap = self.db_dir / self.snapshot
            if not snap.exists():
                raise StoreCorrupt(f"index snapshot {snap} named by {man} is missing")
            engine.index_load(str(snap))
            self.snapshot_bytes = snap.stat().st_size
        jpath = self.db_dir / self.journal
        entries, valid = read_journal(jpath)
        if jpath.exists() and valid < jpath.stat().st_size:
            logger.warning("index journal %s: dropping a torn tail of %d bytes", jpath,
                           jpath.stat().st_size - valid)
            with open(jpath, "r+b") as f:
                f.truncate(valid)
                f.flush()
                os.fsync(f.fileno())
        self.journal_bytes = valid
        for op, track, _name, _recs in entries:
            if op == OP_STORE:
                nxt = max(nxt, track + 1)
        self.loaded = True
        return ids, nxt, entries

    # -- journal appends --
    def _append(self, blob: bytes) -> None:
        if not self.loaded:
            raise RuntimeError("index store appended to before it was loaded")
        self.db_dir.mkdir(parents=True, exist_ok=True)
        path = self.db_dir / self.journal
        new = not path.exists()
        with open(path, "ab") as f:
            if f.tell() != self.journal_bytes:  # a failed earlier append left bytes behind
                f.truncate(self.journal_bytes)
                f.seek(self.journal_bytes)
            f.write(blob)
            f.flush()
            os.fsync(f.fileno())
        if new:
            _fsync_dir(self.db_dir)
        self.journal_bytes += len(blob)

    def append_store(self, track: int, name: str, recs: np.ndarray) -> None:
        self._append(encode_entry(OP_STORE, track, name, recs))

    def append_delete(self, track: int, name: str) -> None:
        self._append(encode_entry(OP_DELETE, track, name))

    # -- checkpoints --
    def should_checkpoint(self) -> bool:
        return self.journal_bytes >= max(self.checkpoint_min_bytes, self.snapshot_bytes)

    def checkpoint(self, engine, ids: dict[str, int], nxt: int) -> None:
        """Compact, snapshot and start an empty journal as generation gen + 1 (one atomic
        manifest replace commits it), then delete the previous generation's files."""
        if not self.loaded:
            raise RuntimeError("index store checkpointed before it was loaded")
        self.db_dir.mkdir(parents=True, exist_ok=True)
        dropped = engine.index_compact()
        g = self.gen + 1
        snap, jour = f"index.{g}.aidfp", f"journal.{g}.aidfj"
        tmp = self.db_dir / (snap + ".tmp")
        engine.index_save(str(tmp))
        with open(tmp, "rb+") as f:
            os.fsync(f.fileno())
        os.replace(tmp, self.db_dir / snap)
        (self.db_dir / jour).unlink(missing_ok=True)
        man = {"version": 2, "gen": g, "snapshot": snap, "journal": jour, "ids": ids, "next": int(nxt)}
        mtmp = self.db_dir / (MANIFEST + ".tmp")
        with open(mtmp, "w") as f:
            f.write(json.dumps(man))
            f.flush()
            os.fsync(f.fileno())
        os.replace(mtmp, self.db_dir / MANIFEST)  # commit point
        _fsync_dir(self.db_dir)
        old = [self.snapshot, self.journal]
        self.gen, self.snapshot, self.journal = g, snap, jour
        self.snapshot_bytes = (self.db_dir / snap).stat().st_size
        self.journal_bytes = 0
        for name in old:
            if name and name not in (snap, jour):
                (self.db_dir / name).unlink(missing_ok=True)
        logger.info("index checkpoint gen %d: %d bytes, %d removed postings compacted", g, self.snapshot_bytes,
                    dropped)

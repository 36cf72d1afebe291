#!/usr/bin/env python3
"""Index an existing audio-ident catalog into the MI355X engine ("Migrating an existing
OLAF_DB"). Olaf's LMDB cannot be read and its hashes are not the engine's, so every Track is stored again
under its own id from its stored raw copy. Run inside the audio-ident service environment (it imports the
service's settings, session factory, Track model and ffmpeg decoder):

    AIDFP_DB=/new/empty/dir python tools/migrate_olaf_db.py --service /path/to/audio-ident-service

The reference's ingest CLI cannot do this: its SHA-256 duplicate check (pipeline.py:102-120) skips
every file Postgres already holds.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))


async def migrate(limit: int | None) -> int:
    from sqlalchemy import select

    from aidfp import fingerprint as fp
    from app.audio.decode import decode_to_pcm  # decode.py:17-71 (ffmpeg, 16 kHz mono f32le)
    from app.db.session import async_session_factory
    from app.models.track import Track

    svc = fp.get_service()
    svc.persist = False  # bulk: no per-track journal fsync; one checkpoint below
    done = failed = 0
    async with async_session_factory() as session:
        rows = (await session.execute(select(Track.id, Track.file_path))).all()
    for tid, path in rows[:limit]:
        try:
            pcm = await decode_to_pcm(Path(path).read_bytes(), 16000)
            ok = await fp.olaf_index_track(pcm, tid)
        except Exception:  # one unreadable file does not stop the migration
            logging.exception("track %s (%s) not indexed", tid, path)
            ok = False
        done += ok
        failed += not ok
    svc.checkpoint()
    svc.persist = True
    logging.info("indexed %d tracks, %d failed", done, failed)
    return 0 if failed == 0 else 1


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--service", required=True, help="audio-ident-service directory (its `app` package)")
    ap.add_argument("--limit", type=int, default=None)
    args = ap.parse_args()
    sys.path.insert(0, str(Path(args.service).resolve()))
    logging.basicConfig(level=logging.INFO)
    return asyncio.run(migrate(args.limit))


if __name__ == "__main__":
    sys.exit(main())

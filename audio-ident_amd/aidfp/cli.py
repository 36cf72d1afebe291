"""`olaf_c`-compatible command line over the GPU engine.

    python -m aidfp.cli store <file.raw> <name>
    python -m aidfp.cli query <file.raw> query
    python -m aidfp.cli del <name>

with the index directory in env OLAF_DB, exactly the invocation the reference
makes (audio-ident-service/app/audio/fingerprint.py:117-125, 185-193, 239-246):
raw 16 kHz mono f32le input, exit code 0 on success, query results on stdout as
`match_count, q_start, q_stop, ref_path, ref_id, ref_start, ref_stop` lines.
Point settings.olaf_bin_path at the `aidfp_olaf_c` wrapper to
swap engines without editing the service.
"""

from __future__ import annotations

import sys
from pathlib import Path

from .fingerprint import FingerprintService, OlafError, db_path, format_match


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("store", "query", "del"):
        print("usage: aidfp.cli store <raw> <name> | query <raw> query | del <name>", file=sys.stderr)
        return 2
    svc = FingerprintService(db_path())
    try:
        if argv[0] == "store" and len(argv) >= 3:
            ok = svc.index_track(Path(argv[1]).read_bytes(), argv[2])
        elif argv[0] == "query" and len(argv) >= 2:
            for m in svc.query(Path(argv[1]).read_bytes()):
                print(format_match(m))
            ok = True
        elif argv[0] == "del" and len(argv) >= 2:
            ok = svc.delete_track(argv[1])
        else:
            print(f"bad arguments: {argv}", file=sys.stderr)
            return 2
    except (OlafError, OSError) as exc:
        print(str(exc), file=sys.stderr)
        return 1
    finally:
        svc.close()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

"""Fold scripts/sessions/<round>*.sh into scripts/ARCHIVE.md and remove them.

    python scripts/archive_sessions.py r06 <commit-that-still-has-them>

Each script becomes one table row: its name and its header comment (the
lines after the shebang up to the first command). The scripts themselves
stay in git history at the named commit."""
import glob
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def header(path):
    words = []
    with open(path) as f:
        for line in f.readlines()[1:]:
            if not line.startswith("#"):
                break
            words.append(line[1:].strip())
    return " ".join(w for w in words if w) or "(no header comment)"


def main():
    rnd, commit = sys.argv[1], sys.argv[2]
    paths = sorted(glob.glob(os.path.join(HERE, "sessions", f"{rnd}*.sh")))
    if not paths:
        raise SystemExit(f"no scripts/sessions/{rnd}*.sh")
    rows = [f"| `{os.path.basename(p)}` | {header(p).replace('|', '/')} |" for p in paths]
    archive = os.path.join(HERE, "ARCHIVE.md")
    if f"## {rnd} sessions" in open(archive).read():
        # a later batch of the same round: rows appended to its table (the
        # round's section is the file's last), the commit named with them
        with open(archive, "a") as f:
            f.write("\n".join(r[:-1] + f" (commit `{commit}`) |" for r in rows) + "\n")
        for p in paths:
            os.remove(p)
        print(f"archived {len(paths)} scripts")
        return
    text = (f"\n## {rnd} sessions (removed at the end of {rnd})\n\n"
            f"The {rnd} `gpurun` command lists; each is in git history at commit "
            f"`{commit}` (`git show {commit}:scripts/sessions/<name>`). The records they "
            f"wrote are under `profiles/{rnd}_*` (`profiles/README.md` names the session "
            f"behind each folder by its letter).\n\n| script | what it ran |\n|---|---|\n"
            + "\n".join(rows) + "\n")
    with open(os.path.join(HERE, "ARCHIVE.md"), "a") as f:
        f.write(text)
    for p in paths:
        os.remove(p)
    print(f"archived {len(paths)} scripts")


if __name__ == "__main__":
    main()

"""One-off assembly of round 5's DESIGN.md from its parts (kept for the record of how
the current-results sections were produced: every table in §5 / §6 comes from
tools/design_tables.py over one tag's committed profiles).
Usage: python tools/assemble_design.py <tag> <main.md> <hostpath.md> <next.md> <appendix.md> <extra_results.md>
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, main_md, host_md, next_md, app_md, extra_md = sys.argv[1:7]
    tables = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "design_tables.py"), tag],
                            capture_output=True, text=True, check=True).stdout
    # split the generated sections: device results (§5) and the drop-in table (§6)
    marker = "### Per-object drop-in"
    dev, _, drop = tables.partition(marker)
    drop_table = "\n".join(ln for ln in drop.splitlines()[1:] if ln.strip())
    main = open(main_md).read()
    host = open(host_md).read().replace("DROPIN_TABLE", drop_table)
    extra = open(extra_md).read()
    main = main.replace("RESULTS_PLACEHOLDER", extra.split("HOST_SECTION")[0].strip() + "\n\n" + dev.strip())
    host = host.replace("DROPIN_TEXT", extra.split("HOST_SECTION")[1].split("DROPIN_END")[0].strip())
    host = host.replace("HOST_TABLE", extra.split("DROPIN_END")[1].strip())
    main = main.replace("HOSTPATH_PLACEHOLDER", host.strip())
    main = main.replace("NEXT_PLACEHOLDER", open(next_md).read().strip())
    main = main.replace("profiles/DROPIN_LOG", f"profiles/{tag}_drop_in.log")
    with open(os.path.join(ROOT, "DESIGN.md"), "w") as f:
        f.write(main.rstrip() + "\n" + open(app_md).read())


if __name__ == "__main__":
    main()

"""Extract the table-driven golden vectors of the reference's state-machine tests.

Source: /root/reference/src/state_machine_tests.zig. Each `try check(...)` call there holds one
table written in the row DSL of src/testing/table.zig: every row is an input event plus its
expected result (`account ... created`, `transfer ... exceeds_credits`, `lookup_account A1 0 15 0 0
_`, ...). This script copies only those table rows (data: inputs and expected outputs) into
tests/golden/tables/<test-slug>__<n>.txt; it copies no test logic. Zig `//` comment lines between
rows are dropped; trailing `// ...` row comments are kept (the DSL ignores them).

Run in the build container (the reference is not present on the GPU box):
    python tests/golden/extract_tables.py
"""
import json
import os
import re
import sys

REFERENCE = "/root/reference/src/state_machine_tests.zig"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tables")


def slug(name: str) -> str:
    s = re.sub(r"[^A-Za-z0-9]+", "_", name).strip("_").lower()
    return s or "table"


def extract(path: str):
    lines = open(path, encoding="utf-8").read().split("\n")
    tables = []
    test_name = None
    in_check = False
    rows = []
    start_line = 0
    for lineno, line in enumerate(lines, 1):
        m = re.match(r'^test "(.*)" \{', line)
        if m:
            test_name = m.group(1)
            continue
        stripped = line.strip()
        if stripped.startswith("try check("):
            in_check = True
            rows = []
            start_line = lineno
            continue
        if in_check:
            if stripped.startswith("\\\\"):
                rows.append(stripped[2:].strip())
            elif stripped.startswith(");"):
                in_check = False
                tables.append((test_name, start_line, [r for r in rows]))
    return tables


def main():
    if not os.path.exists(REFERENCE):
        sys.exit(f"reference not found: {REFERENCE}")
    os.makedirs(OUT, exist_ok=True)
    index = []
    counts = {}
    for name, line, rows in extract(REFERENCE):
        base = slug(name)
        counts[base] = counts.get(base, 0) + 1
        fname = f"{base}__{counts[base]}.txt"
        with open(os.path.join(OUT, fname), "w") as f:
            f.write(f"# test \"{name}\" (src/state_machine_tests.zig:{line})\n")
            for r in rows:
                f.write(r + "\n")
        index.append({"file": fname, "test": name, "line": line, "rows": len(rows)})
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump(index, f, indent=1)
    print(f"wrote {len(index)} tables to {OUT}")


if __name__ == "__main__":
    main()

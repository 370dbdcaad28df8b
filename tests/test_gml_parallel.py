"""The GML reader's parallel graph list (gml.c parse_graph_parallel): a large file's node/edge
items are parsed in pieces on several threads and concatenated in file order. The result must be
the one-thread parse's in every field -- vertex and edge order, endpoints, attribute names, types
(string if any element, in any piece, gives a string) and values, `directed` (the last one wins),
and the error message with its line when the file is bad. tests/gml_parallel_check.c parses each
file both ways (gml_parse_ex with par_min = 0) and compares; it prints the number of pieces the
parallel parse used, so the cases that must take it (and the ones that must fall back) are
checked too. CPU only."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "shadow_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("gml") / "gml_parallel_check")
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-I" + SRC, "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "gml_parallel_check.c"), os.path.join(SRC, "gml.c"),
                    "-o", exe, "-lpthread", "-lm"], check=True)
    return exe


def _run(checker, tmp_path, text, threads):
    p = tmp_path / "g.gml"
    p.write_text(text)
    r = subprocess.run([checker, str(p), str(threads)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout.split()


def _graph(n, m, seed, mixed=True, extra=""):
    rng = random.Random(seed)
    out = ["# generated", "Creator \"test\"", "graph [", "  directed 1", "  label \"g\""]
    for v in range(n):
        items = [f"    id {v * 3 + 7}", f"    label \"h{v}\""]
        if rng.random() < 0.7:
            items.append(f"    host_bandwidth_up {rng.randint(1, 10**6)}")
        if mixed and v > n // 2 and rng.random() < 0.1:
            items.append("    ip_address \"11.0.0.%d\"" % (v % 250))
        elif rng.random() < 0.5:
            items.append(f"    ip_address {v}")  # numeric here, a string later: string overall
        if rng.random() < 0.2:
            items.append("    graphics [ x 1.5 y -2 label \"n\" ]")
        if rng.random() < 0.05:
            items.append("    # a comment line")
        out.append("  node [\n" + "\n".join(items) + "\n  ]")
        if v == n // 3:
            out.append("  directed 0")
    for e in range(m):
        a, b = rng.randrange(n), rng.randrange(n)
        items = [f"    source {a * 3 + 7}", f"    target {b * 3 + 7}",
                 f"    latency \"{rng.randint(1, 90)} ms\""]
        if rng.random() < 0.8:
            items.append(f"    packet_loss {rng.randint(0, 50) / 1000.0}")
        if e == m // 2:
            items.append("    note \"a &amp; b\"")
        out.append("  edge [ " + " ".join(items) + " ]" if e % 3 == 0 else "  edge [\n" + "\n".join(items) + "\n  ]")
    out.append("]")
    out.append(extra)
    return "\n".join(out) + "\n"


@pytest.mark.parametrize("threads", [2, 4, 8])
def test_parallel_gml_matches_one_thread(checker, tmp_path, threads):
    out = _run(checker, tmp_path, _graph(3000, 12000, 11 + threads), threads)
    assert out[0] == "same", out
    assert int(out[1]) == 3000 and int(out[2]) == 12000
    assert int(out[3]) > 1, out  # the pieces path ran


def test_parallel_gml_trailing_lists_and_second_graph(checker, tmp_path):
    extra = "other [ a 1 b [ c 2 ] ]\ngraph [ node [ id 1 ] ]\nversion 3\n"
    out = _run(checker, tmp_path, _graph(1500, 4000, 5, extra=extra), 4)
    assert out[0] == "same" and int(out[3]) > 1, out


def test_parallel_gml_falls_back_on_item_lookalike_in_string(checker, tmp_path):
    """a quoted string spanning lines that holds `edge [` at a line start: the piece before it
    does not stop on that candidate, so the list is parsed by one thread"""
    g = _graph(800, 2400, 7).split("\n")
    cut = len(g) // 2
    g.insert(cut, "  note \"first line\n  edge [ source 7 target 10 ]\n  node [ id 99999 ]\nlast\"")
    text = "\n".join(g)
    for t in (2, 3, 4, 8):
        out = _run(checker, tmp_path, text, t)
        assert out[0] == "same", out


@pytest.mark.parametrize("bad", ["unknown_id", "bad_token", "unterminated", "late_error"])
def test_parallel_gml_errors_match_one_thread(checker, tmp_path, bad):
    text = _graph(1200, 3000, 3)
    if bad == "unknown_id":
        i = text.index("source ", len(text) // 2)  # an id no node has (ids are 7, 10, 13, ...)
        j = text.index("\n" if text[i:].split("\n", 1)[0].count("target") == 0 else " target", i)
        text = text[:i] + "source 4" + text[j:]
    elif bad == "bad_token":
        lines = text.split("\n")
        lines[len(lines) * 2 // 3] += " @@"
        text = "\n".join(lines)
    elif bad == "unterminated":
        text = text.rstrip().rstrip("]")
    else:  # an error after the graph list: the message's line comes from the one-thread parse
        text += "tail [ x ]\n  ?\n"
    out = _run(checker, tmp_path, text, 4)
    assert out[0] == "same-error", out

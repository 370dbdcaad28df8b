"""Writes a large synthetic Shadow-style GML (nodes with bandwidth strings, edges with latency
strings and packet_loss) for timing the GML reader: python tools/gml_big.py OUT [nodes] [edges]"""
import random
import sys

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
m = int(sys.argv[3]) if len(sys.argv) > 3 else 2000000
rng = random.Random(1)
with open(out, "w") as f:
    f.write("graph [\n  directed 0\n")
    for v in range(n):
        f.write(f'  node [\n    id {v}\n    host_bandwidth_up "{rng.randint(1, 10**6)} Kibit"\n'
                f'    host_bandwidth_down "{rng.randint(1, 10**6)} Kibit"\n  ]\n')
    for e in range(m):
        f.write(f"  edge [\n    source {rng.randrange(n)}\n    target {rng.randrange(n)}\n"
                f'    latency "{rng.randint(1, 200)} ms"\n    packet_loss {rng.randint(0, 50) / 1000.0}\n  ]\n')
    f.write("]\n")

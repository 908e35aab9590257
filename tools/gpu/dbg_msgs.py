"""Debug aid: record sequences of the GPU and oracle partitions for a small C5-shape run (prints differences)."""
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import msgpack

from test_gpu_messages import catch_workflow, clusters

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
gpu, ref, cg, co = clusters(P, catch_workflow())
for i in range(n):
    gpu[i % P].create("wf", [msgpack.packb({"orderId": "order-%d" % i})])
    ref[i % P].create("wf", msgpack.packb({"orderId": "order-%d" % i}))
cg.settle()
co.settle()
if len(sys.argv) > 3:
    cks = [b"order-%d" % i for i in range(n)]
    pls = [msgpack.packb({"foo": i}) for i in range(n)]
    cg.publish(b"order canceled", cks, pls)
    print("gpu published; pending", [(g.pending(1), g.pending(2)) for g in gpu], flush=True)
    co.publish(b"order canceled", cks, pls)
print("rounds", cg.rounds, co.rounds)
for p in range(P):
    a, b = ref[p].records(), gpu[p].records()
    print("partition", p, len(a), len(b))
    from collections import Counter
    print("oracle", sorted(Counter((x.record_type, x.value_type, x.intent) for x in a).items()))
    print("gpu   ", sorted(Counter((x.record_type, x.value_type, x.intent) for x in b).items()))
    shown = 0
    for k in range(max(len(a), len(b))):
        x = a[k] if k < len(a) else None
        y = b[k] if k < len(b) else None
        fx = (x.position, x.key, x.record_type, x.value_type, x.intent) if x else None
        fy = (y.position, y.key, y.record_type, y.value_type, y.intent) if y else None
        if fx != fy or n <= 4:
            print("%6d %s %-40s %-40s" % (k, "  " if fx == fy else "!!", fx, fy))
            shown += 1
            if shown > 60:
                break

"""Static instruction mix of one kernel in a hipcc -S listing.
usage: python scripts/isa_count.py file.s 'k_safe_step<0,0,1>' [top]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
want = sys.argv[2]
m = re.match(r"(\w+)<(.*)>", want)
name, targs = m.group(1), [int(t) for t in m.group(2).split(",")]
mangled = "k_safe_step" if False else name
pat = "%d%s" % (len(name), name) + "IL" + "EL".join("i%d" % t for t in targs).replace("i", "i") + "E"
sym = None
for cand in re.findall(r"^(_Z\S+):", s, re.M):
    if ("%d%s" % (len(name), name)) in cand and re.search("I" + "".join("L[ib]%dE" % t for t in targs) + "E", cand):
        sym = cand
        break
if sym is None:
    sys.exit("kernel not found")
body = s[s.index(sym + ":"):]
body = body[: body.index(".Lfunc_end")]
ins = [l.strip().split()[0] for l in body.split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = Counter(ins)
valu = sum(v for k, v in c.items() if k.startswith("v_"))
f64 = sum(v for k, v in c.items() if k.startswith("v_") and "f64" in k)
vm = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))
print(sym[:70], "total", len(ins), "valu", valu, "f64", f64, "vmem", vm, "salu", sum(v for k, v in c.items() if k.startswith("s_")))
print(c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40))

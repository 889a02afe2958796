import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    c3 = [x.get('c3_us', 0) for x in v]; c2 = [x.get('c2_us', 0) for x in v]
    print(f"{k.split('/')[-1]:28s} c3 {sorted(c3)[len(c3)//2]:7.1f} {[round(x,1) for x in c3]}  c2 {sorted(c2)[len(c2)//2]:6.1f}")

import json, collections, sys
ops=json.load(open(sys.argv[1]))
tot=sum(o['ms'] for o in ops)
print("total ms", round(tot,3), "n", len(ops))
cat=collections.defaultdict(lambda:[0,0,0])
for o in ops:
    l=o['op']
    k = 'convT' if 'upsample' in l else ('stem' if 'projection_layer.0' in l and 'dla_down' in l else ('heads' if l.startswith('heads') else ('block0' if 'block_layers.0' in l else ('prep' if 'staging' in l else 'other'))))
    cat[k][0]+=o['ms']; cat[k][1]+=o['gflop']; cat[k][2]+=1
for k,v in cat.items(): print(f"{k:8s} {v[0]:7.3f} ms {v[1]:8.1f} GF {v[2]:3d} ops {v[1]/max(v[0],1e-9):7.1f} TF")

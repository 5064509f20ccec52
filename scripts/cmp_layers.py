import json,sys
a=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], a['sum_ms'], sys.argv[2], b['sum_ms'])
for x,y in zip(a['layers'],b['layers']):
    if abs(x['ms']-y['ms'])>0.003: print(x['layer'], x['shape'], x['ms'], y['ms'])

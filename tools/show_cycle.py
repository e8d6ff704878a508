import csv, collections, json, sys
T = sys.argv[1]
print(open(f'gpurun_out/t_{T}.log').read().strip().splitlines()[-1])
d = json.load(open(f'gpurun_out/bench_{T}.json'))
print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'ms/step', d['ms_per_step'])
print(''.join(open(f'gpurun_out/stamps_{T}.txt').read().strip().splitlines(True)[-5:]))
rows = list(csv.DictReader(open(f'gpurun_out/pmc_{T}/pmc_counter_collection.csv')))
agg = collections.defaultdict(float); cnt = collections.Counter()
for r in rows:
    if 'env_step' in r['Kernel_Name']:
        agg[r['Counter_Name']] += float(r['Counter_Value']); cnt[r['Counter_Name']] += 1
print({k: round(v / cnt[k] / 4096, 1) for k, v in sorted(agg.items())})

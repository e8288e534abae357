import json
for f in ['bs', 'bo']:
    d = json.load(open('gpurun_out/' + f + '.json'))
    print(f, d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms_per_step'].items() if k != 'launches'})

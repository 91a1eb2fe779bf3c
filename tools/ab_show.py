import json, glob, sys
for f in sorted(glob.glob('gpurun_out/ablib/*.json')):
    try:
        d = json.loads(open(f).read())
        print(f.split('/')[-1], d['value'], d['enc_kernel_us'], d['dec_kernel_us'], d.get('device_error'))
    except Exception as e:
        print(f, 'bad', e)

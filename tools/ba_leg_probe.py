import sys, time, json
sys.path.insert(0, '/root/repo')
import bench
print(json.dumps({k: v for k, v in bench.localba_leg(0, calls=8, cpu=False).items() if k != 'roofline'}))
print(json.dumps({k: v for k, v in bench.localba_leg(0, calls=30, cpu=False).items() if k != 'roofline'}))

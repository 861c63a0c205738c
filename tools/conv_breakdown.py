import csv, sys
sys.path.insert(0,'/root/repo/fast-cwdm_amd')
rows=[r for r in csv.DictReader(open(sys.argv[1])) if ('conv3d_kernel' in r['Kernel_Name'] or 'conv3d_wide_kernel' in r['Kernel_Name'])]
# last forward = last 72 conv launches
last=rows[-72:]
from cwdm_hip.unet_runtime import UNetPlan
import ctypes
# reconstruct conv list from the plan via oracle topology
from oracle import unet as ou
blocks = ou.topology()
convs=[]
lvl=0
for b in blocks:
    if b['kind']=='conv_in': convs.append(('conv_in',0,b['cin'],b['cout'],0)); continue
    if b['kind']=='out': convs.append(('out',0,b['cin'],b['cout'],0)); continue
    ud=b['updown']; lo = lvl+1 if ud=='down' else (lvl-1 if ud=='up' else lvl)
    convs.append((b['prefix']+'.c1',lo,b['cin'],b['cout'],0))
    convs.append((b['prefix']+'.c2',lo,b['cout'],b['cout'], b['cin'] if b['cin']!=b['cout'] else 0))
    lvl=lo
n=int(sys.argv[2]) if len(sys.argv)>2 else 128
tot=0; totf=0
for (name,l,ci,co,cb),r in zip(convs,last):
    dt=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    v=(n>>l)**3
    fl=2*v*co*(27*ci+cb)
    tot+=dt; totf+=fl
    print(f"{name:28s} L{l} {ci:4d}->{co:4d} {dt:9.1f}us {fl/dt/1e6:8.1f}TF/s grid={r['Grid_Size_X']}")
print(tot, totf/tot/1e6)

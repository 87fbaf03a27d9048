import os, sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
import mantis_amd as M
from mantis_amd import synth
W,H,CAMS,RIGS,ND=1280,720,4,256,64
white,red,green=synth.load_map(); K,D=synth.intrinsics(W,H)
rng=np.random.default_rng(1000); ext=synth.rig_extrinsics(CAMS)
cams,Tbc=[],[]
for r in range(ND):
    Twb=synth.random_base_pose(rng)
    for c in range(CAMS):
        Twc=Twb@ext[c]; cams.append(synth.make_cam(Twc[:3,:3],Twc[:3,3],W,H)); Tbc.append(ext[c])
for segm in sys.argv[1:]:
    os.environ['MANTIS_SEG_M']=segm
    m=M.Mantis(max_cams=RIGS*CAMS,max_width=W,max_height=H, max_contour_points=98304)
    m.set_map(white,red,green)
    fb=W*H*3; dev=m.device_alloc(len(cams)*fb); m.synth_render(cams,[synth.frame_seed(3,i) for i in range(len(cams))],dev); m.synchronize()
    imgs=[M.make_image(None,K,D,T_base_cam=Tbc[i%len(cams)],device_ptr=dev+(i%len(cams))*fb,width=W,height=H) for i in range(RIGS*CAMS)]
    b=M.Batch(m,imgs,RIGS); b.run(); m.set_profiling(True); b.run(); kt=dict(m.stage_times()); m.set_profiling(False)
    fc=np.array([m.frame_counters(i)[:24] for i in range(RIGS*CAMS)])
    print("M",segm,"border_trace ms",round(kt.get('border_trace',0),3),"steps_max med/max",int(np.median(fc[:,18])),fc[:,18].max(),"steps_sum med",int(np.median(fc[:,20])),"ticks(us) med/max",np.median(fc[:,21])/100,fc[:,21].max()/100,"chunks med",int(np.median(fc[:,19])),"segs med",int(np.median(fc[:,22])),"overflow",int((fc[:,8]!=0).sum()))
    m.close()

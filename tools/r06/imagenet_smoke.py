import base64, io, time, numpy as np, concurrent.futures as cf
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import seldon_core_amd as sca
from PIL import Image
rng=np.random.default_rng(0)
def png(h,w,seed):
    img=(np.random.default_rng(seed).random((h,w,3))*255).astype(np.uint8)
    b=io.BytesIO(); Image.fromarray(img).save(b,format="PNG"); return b.getvalue()
P=lambda n,v,t="INT": {"name":n,"value":str(v),"type":t}
graph={"name":"ot","type":"OUTPUT_TRANSFORMER","implementation":"IMAGENET_OUTPUT_TRANSFORMER","children":[
 {"name":"it","type":"TRANSFORMER","implementation":"IMAGENET_TRANSFORMER","parameters":[P("size",64)],"children":[
  {"name":"comb","type":"COMBINER","implementation":"IMAGENET_COMBINER","children":[
    {"name":"m1","type":"MODEL","implementation":"IMAGENET_MODEL","parameters":[P("arch","densenet169","STRING"),P("image",64),P("device",-1)]},
    {"name":"m2","type":"MODEL","implementation":"IMAGENET_MODEL","parameters":[P("arch","resnet50","STRING"),P("image",64),P("device",-1)]}]}]}]}
dep=sca.Deployment({"name":"p","graph":graph,"componentSpecs":[{"spec":{"containers":[]}}]}, device=-1)
try:
    req={"binData": base64.b64encode(png(80,90,1)).decode()}
    t=time.time(); out=dep.predict(req); print(out, time.time()-t)
    with cf.ThreadPoolExecutor(8) as ex:
        outs=list(ex.map(lambda i: dep.predict({"binData": base64.b64encode(png(80,90,i)).decode()}), range(16)))
    print([o.get("strData") for o in outs])
    print(dep.engine.unit_kind("m1") if hasattr(dep.engine,'unit_kind') else '')
finally:
    dep.close()

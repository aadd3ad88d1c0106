mkdir -p gpurun_out
python -c "
import subprocess,sys
sys.path.insert(0,'.')
from kubeoperator_amd.control.domain import hosts
r=subprocess.run(['bash','-o','pipefail','-c',hosts.GPU_PROBE],capture_output=True,text=True)
open('gpurun_out/probe_raw.txt','w').write(r.stdout+'\n--stderr--\n'+r.stderr)
" ; ls /sys/class/kfd/kfd/topology/nodes/ > gpurun_out/kfd_ls.txt 2>&1; for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "== $n"; cat $n/properties; cat $n/gpu_id; done > gpurun_out/kfd_props.txt 2>&1; true

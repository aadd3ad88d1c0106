#!/usr/bin/env bash
# KubeOperator-AMD installer (reference scripts/0_prepare.sh … 8_check_install_env.sh + kubeopsctl.sh,
# re-done for an Ubuntu/RHEL controller; the controller itself needs no GPU).
#
#   scripts/install.sh [--mode compose|systemd] [--prefix /opt/kubeoperator] [--check-only]
#
# compose : build the server image and run nginx + server + webkubectl with docker compose
# systemd : install the Python package into a venv under PREFIX and run `kubeopsctl start all` as a unit
set -euo pipefail

MODE=systemd
PREFIX=/opt/kubeoperator
CHECK_ONLY=0
while [[ $# -gt 0 ]]; do
  case "$1" in
    --mode) MODE=$2; shift 2 ;;
    --prefix) PREFIX=$2; shift 2 ;;
    --check-only) CHECK_ONLY=1; shift ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
done
SRC=$(cd "$(dirname "$0")/.." && pwd)

log() { printf '\033[1;32m==>\033[0m %s\n' "$*"; }
die() { printf '\033[1;31mERROR:\033[0m %s\n' "$*" >&2; exit 1; }

check_env() {
  # reference 8_check_install_env.sh: root, >= 2 CPU, >= 8 GB RAM, >= 50 GB free under the install prefix
  [[ $(id -u) -eq 0 ]] || die "run as root"
  local cpus mem_kb free_kb os
  cpus=$(nproc)
  mem_kb=$(awk '/MemTotal/ {print $2}' /proc/meminfo)
  mkdir -p "$PREFIX"
  free_kb=$(df -Pk "$PREFIX" | awk 'NR==2 {print $4}')
  os=$(. /etc/os-release && echo "$ID $VERSION_ID")
  log "controller: $os, $cpus CPUs, $((mem_kb / 1024 / 1024)) GiB RAM, $((free_kb / 1024 / 1024)) GiB free in $PREFIX"
  (( cpus >= 2 )) || die "need >= 2 CPUs"
  (( mem_kb >= 7 * 1024 * 1024 )) || die "need >= 8 GB RAM"
  (( free_kb >= 50 * 1024 * 1024 )) || die "need >= 50 GB free under $PREFIX"
  command -v python3 >/dev/null || die "python3 is required"
  python3 -c 'import sys; sys.exit(0 if sys.version_info >= (3, 10) else 1)' || die "python >= 3.10 required"
  command -v ssh >/dev/null || die "openssh-client is required (provisioning transport)"
  if [[ $MODE == compose ]]; then
    command -v docker >/dev/null || die "docker is required for --mode compose"
    docker compose version >/dev/null 2>&1 || die "docker compose plugin is required"
  fi
  command -v terraform >/dev/null || log "terraform not found: AUTOMATIC (vSphere/OpenStack) plans will be unavailable"
}

install_systemd() {
  log "installing into $PREFIX"
  mkdir -p "$PREFIX"/{conf,data/packages}
  rsync -a --delete --exclude '.git' --exclude 'gpurun_out' "$SRC/kubeoperator_amd" "$PREFIX/"
  [[ -f $PREFIX/conf/config.yml ]] || sed "s#/var/lib/kubeoperator#$PREFIX/data#" "$SRC/conf/config.yml" > "$PREFIX/conf/config.yml"
  python3 -m venv "$PREFIX/venv"
  "$PREFIX/venv/bin/pip" install --quiet -r "$SRC/docker/server/requirements.txt"
  sed -e "s#/usr/bin/python3#$PREFIX/venv/bin/python#g" -e "s#/opt/kubeoperator#$PREFIX#g" \
    "$SRC/scripts/kubeops.service" > /etc/systemd/system/kubeops.service
  cat > /usr/local/bin/kubeopsctl <<EOS
#!/usr/bin/env bash
export KUBEOPERATOR_CONFIG=$PREFIX/conf/config.yml PYTHONPATH=$PREFIX
exec $PREFIX/venv/bin/python -m kubeoperator_amd.control.cli "\$@"
EOS
  chmod +x /usr/local/bin/kubeopsctl
  KUBEOPERATOR_CONFIG=$PREFIX/conf/config.yml PYTHONPATH=$PREFIX "$PREFIX/venv/bin/python" -m kubeoperator_amd.control.cli init
  systemctl daemon-reload
  systemctl enable --now kubeops.service
}

install_compose() {
  log "building and starting the compose topology"
  mkdir -p "$SRC/data/packages"
  (cd "$SRC" && docker compose build server && docker compose up -d)
}

check_env
[[ $CHECK_ONLY -eq 1 ]] && { log "environment OK"; exit 0; }
case $MODE in
  systemd) install_systemd ;;
  compose) install_compose ;;
  *) die "unknown mode $MODE" ;;
esac
log "KubeOperator-AMD is starting; UI at http://$(hostname -I | awk '{print $1}')/ui/ (admin / kubeoperator@admin123 -- change it)"

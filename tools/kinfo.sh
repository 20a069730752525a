#!/bin/bash
# Per-kernel VGPR / scratch / occupancy summary of a gfx950 assembly file (hipcc --cuda-device-only -S).
# usage: tools/kinfo.sh file.s
awk '/^_Z[A-Za-z0-9_]*:/{name=$1} /; NumVgprs:/{v=$3} /; ScratchSize:/{sc=$3} /; Occupancy:/{print name, "vgpr="v, "scratch="sc, "occ="$3}' "$1" | sed -e 's/_ZN3ntt6k_passINS_5Eng29ILi\([0-9]*\)ELi\([0-9]*\)EEELi\([0-9]*\)ELi\([0-9]\)ELb\([01]\)ELb\([01]\)E.*:/k_pass<L\1,W\2> logr=\3 kind=\4 fulltw=\5 fast=\6/'

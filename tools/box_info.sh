#!/bin/bash
# Fingerprint of the GPU box (box-to-box spread is large: same-box A/B only)
{
  hostname; grep -m1 "model name" /proc/cpuinfo
  rocm-smi --showproductname --showcomputepartition --showmemorypartition --showmaxpower --showsclkrange --showvbios --showdriverversion 2>&1 | grep "GPU\[0\]\|Driver"
  rocm-smi --showfwinfo 2>&1 | grep "GPU\[0\]" | head -30
  rocminfo 2>/dev/null | awk '/Agent 2/{f=1} f&&/Marketing Name|Compute Unit|Max Clock|L1|L2|L3|Cache Info|Chip ID|ASIC Revision|Memory Properties|SIMDs per CU|Shader Engines/{print}' | head -20
  cat /sys/class/drm/card*/device/current_link_speed 2>/dev/null | head -2
} 2>&1

#!/bin/bash
# print VGPR / scratch / occupancy per kernel of every libmpfft translation unit
for f in mpir-fft_amd/csrc/*.hip; do
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -o /tmp/_regs.o $f -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: //; s/ \[-Rpass.*//' | paste - - - - \
 | sed -E 's/Function Name: //; s/VGPRs: //; s/ScratchSize \[bytes\/lane\]: //; s/Occupancy \[waves\/SIMD\]: //' | awk '{printf "%-45s vgpr=%-4s scratch=%-4s occ=%s\n", $1, $2, $3, $4}'
done

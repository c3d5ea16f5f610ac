#!/bin/bash
# torchrun --no-python wrapper: rank 0 runs under rocprofv3 counter
# collection (counters $PMC into $PMC_DIR), the other ranks run plainly.
# TCC counters are device-wide: rank 0's dispatch windows also count the
# other ranks' traffic on the shared card.
if [ "$RANK" = "0" ]; then
  exec rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d "$PMC_DIR" -o run -- python "$@"
else
  exec python "$@"
fi

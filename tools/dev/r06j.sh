#!/bin/bash
# (1) end-to-end leg under SDMA settings (which copy engine the runtime uses); (2) config #3 with a
# bigger deep budget / other tier-0 table sizes.
bash tools/dev/r06h.sh && bash tools/dev/r06i.sh

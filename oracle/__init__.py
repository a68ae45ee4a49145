"""CPU restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY (see thunder_oracle.h)."""

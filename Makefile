# Builds the MI355X (gfx950) library and the CPU oracle.
#   make            -> adversarial_learning_on_pointclouds_amd/lib/libpcadv.so
#   make asm        -> kernel assembly + resource usage under build/
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := adversarial_learning_on_pointclouds_amd
SRC := $(wildcard $(PKG)/csrc/*.hip)
CPP := $(wildcard $(PKG)/csrc/*.cpp)
OBJ := $(patsubst $(PKG)/csrc/%.hip,build/obj/%.o,$(SRC)) $(patsubst $(PKG)/csrc/%.cpp,build/obj/%.host.o,$(CPP))
HDR := $(wildcard $(PKG)/csrc/*.h) include/pcadv.h
LIB := $(PKG)/lib/libpcadv.so
HIPFLAGS := -O3 --offload-arch=$(ARCH) -fPIC -std=c++17 -Wall -Wno-unused-function -Iinclude

all: $(LIB)

build/obj/%.o: $(PKG)/csrc/%.hip $(HDR)
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only C++ (the dataset reader)
build/obj/%.host.o: $(PKG)/csrc/%.cpp $(HDR)
	@mkdir -p build/obj
	$(HIPCC) -O2 -fPIC -std=c++17 -Wall -Iinclude -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p $(PKG)/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ) -lz

asm: $(SRC)
	@mkdir -p build/asm
	for f in $(SRC); do $(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage --cuda-device-only -S $$f -o build/asm/$$(basename $$f .hip).s 2> build/asm/$$(basename $$f .hip).usage; done

clean:
	rm -rf build $(LIB)

.PHONY: all asm clean

# diagnostic build with per-phase timestamps (never loaded by the product path)
STAMPS_LIB := build/stamps/libpcadv_stamps.so
stamps: $(SRC) $(HDR)
	@mkdir -p build/stamps
	$(HIPCC) $(HIPFLAGS) -DPCADV_STAMPS -shared -o $(STAMPS_LIB) $(SRC) $(CPP) -lz
.PHONY: stamps

# A/B variant library (tools/gpu_ab.sh): the same sources with ABDEFS, e.g.
#   make ab ABDEFS=-DPCADV_K2_PRIO=0
ABDEFS ?=
ab: $(SRC) $(HDR)
	@mkdir -p build/ab
	$(HIPCC) $(HIPFLAGS) $(ABDEFS) -shared -o build/ab/libA.so $(SRC) $(CPP) -lz
.PHONY: ab

# AddressSanitizer + UBSan host build of the HDF5 reader with a small driver
# (tests/test_h5_asan.py feeds it truncated / corrupted files)
ASAN_BIN := build/asan/h5check
asan: $(ASAN_BIN)
$(ASAN_BIN): $(PKG)/csrc/h5read.cpp tests/asan/h5check.cpp include/pcadv.h
	@mkdir -p build/asan
	g++ -std=c++17 -g -O1 -fsanitize=address,undefined -fno-omit-frame-pointer \
	  -fno-sanitize-recover=undefined -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude \
	  $(PKG)/csrc/h5read.cpp tests/asan/h5check.cpp -lz -o $@.tmp.$$$$ && mv -f $@.tmp.$$$$ $@
.PHONY: asan

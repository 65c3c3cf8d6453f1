# Builds the UNMODIFIED reference Fortran (read in place from $(REF)) with AMD flang
# into oracle/_ref/ only.  Test infrastructure: used to generate and pin the golden
# fixtures under tests/golden/ and, optionally, as the "reference" CPU baseline.
# Nothing here is shipped or linked by the product.
#
#   make -f oracle/ref.mk            (from the repo root)
#
# Build mode: the reference's own default macros (macros/mpp_macros.fi:
# _MPP_BLOCK_MODE_, _DD_MANUAL_BLOCK_GRID_), no GPU macros.  Run it with
# OMP_NUM_THREADS=1 (NO_PARALLEL mode with >1 thread races).
#
# MPI: MPICH 3.3.2 from /opt/conda.  Its mpi.mod is gfortran-format and cannot be
# read by flang, so the `mpi` module is recompiled for flang from MPICH's own
# public mpif.h (mpi_shim.f90 = `module mpi; include 'mpif.h'; end module`;
# shared/mpp/mpp.f90:17 carries the same include, commented out).  The library
# linked is MPICH's own libmpi/libmpifort; no reference source is edited or copied.

REF     ?= /root/reference
OUT     ?= oracle/_ref
REFFC   ?= /opt/rocm/lib/llvm/bin/flang
MPIINC  ?= /opt/conda/include
MPILIB  ?= /opt/conda/lib
FFLAGS  ?= -cpp -O2 -fopenmp -fPIC -I$(REF) -I$(REF)/macros -I/opt/rocm/lib/llvm/include/flang -module-dir $(OUT)/mod -I$(OUT)/mod
LDLIBS  ?= -L$(MPILIB) -Wl,-rpath,$(MPILIB) -lmpifort -lmpi -fopenmp

SRCS = shared/kind.f90 shared/system.f90 shared/kernel_runtime.f90 shared/constants.f90 \
       shared/mpp/mpp.f90 shared/errors.f90 shared/debug.f90 shared/mpp/hilbert_curve.f90 \
       legacy/service/input_output_data.f90 legacy/service/rw_ctl_file.f90 \
       legacy/service/read_write_parameters.f90 legacy/service/time_tools.f90 \
       configs/basinpar.f90 configs/sw.f90 configs/parallel.f90 configs/cmd.f90 \
       core/math_tools.f90 core/decomposition.f90 core/data_types.f90 shared/mpp/sync.f90 \
       core/grid.f90 core/ocean.f90 core/kernel_interface.f90 \
       tools/io.f90 tools/time_manager.f90 \
       kernel/shallow_water/depth.f90 kernel/shallow_water/vel_ssh.f90 kernel/shallow_water/mixing.f90 \
       kernel/service/grid_parameters.f90 kernel/service/grid_kernels.f90 kernel/tracer/leapfrog_tracer.f90 \
       interface/shallow_water/sw_interface.f90 interface/service/grid_interface.f90 interface/tracer/tracer_interface.f90 \
       service/gridcon.f90 service/basinpar_construction.f90 \
       control/init_data.f90 control/output.f90 control/shallow_water/shallow_water.f90 \
       control/preprocess.f90 control/tracer.f90

OBJS = $(addprefix $(OUT)/obj/,$(SRCS:.f90=.o))

all: $(OUT)/model $(OUT)/libref.so $(OUT)/ref_driver

$(OUT)/obj/mpi_shim.o: oracle/mpi_shim.f90
	@mkdir -p $(dir $@) $(OUT)/mod
	$(REFFC) $(FFLAGS) -I$(MPIINC) -c -o $@ $<

# Module dependencies follow the reference makefile's source order: build serially.
$(OUT)/.objs: $(OUT)/obj/mpi_shim.o
	@set -e; for s in $(SRCS); do \
	  o=$(OUT)/obj/$${s%.f90}.o; mkdir -p $$(dirname $$o); \
	  $(REFFC) $(FFLAGS) -c -o $$o $(REF)/$$s; done
	@touch $@

$(OUT)/model: $(OUT)/.objs
	$(REFFC) -o $@ $(OUT)/obj/mpi_shim.o $(OBJS) $(REF)/model.f90 $(FFLAGS) $(LDLIBS)

$(OUT)/ref_driver: $(OUT)/.objs oracle/ref_driver.f90
	$(REFFC) -o $@ $(OUT)/obj/mpi_shim.o $(OBJS) oracle/ref_driver.f90 $(FFLAGS) $(LDLIBS)

$(OUT)/libref.so: $(OUT)/.objs
	$(REFFC) -shared -o $@ $(OUT)/obj/mpi_shim.o $(OBJS) $(LDLIBS)

clean:
	rm -rf $(OUT)

.PHONY: all clean

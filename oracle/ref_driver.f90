! ref_driver.f90 -- TEST INFRASTRUCTURE (fixture generator), not product code.
!
! Drives the unmodified, compiled reference (oracle/_ref, see oracle/ref.mk) through
! exactly the init sequence of model.f90:47-91 (mpp_init, basin.par/sw.par/parallel.par,
! read_global_mask, domain init, init_grid_data, init_ocean_data) and then NSTEPS model steps
! (model.f90:146-160: expl_shallow_water(tau), control/shallow_water/shallow_water.f90:22,
! then expl_tracer(tau), control/tracer.f90:33), with tau = 1 s (ocean_run.par line 2).
! Afterwards every field the step touches is dumped, per block, with its bounds, as raw
! little-endian stream records into DUMPFILE (header: block count, tracer count).
!
! usage (in a directory holding basin.par, sw.par, parallel.par):
!     ref_driver NSTEPS DUMPFILE
program ref_driver
    use kind_module, only: wp8 => SHR_KIND_R8, wp4 => SHR_KIND_R4
    use mpp_module
    use config_basinpar_module, only: load_config_basinpar_from_file
    use config_sw_module, only: load_config_sw_from_file, use_tracers, tracer_num
    use config_parallel_module, only: load_config_parallel_from_file_and_cmd
    use decomposition_module, only: domain_data
    use mpp_sync_module, only: mpp_sync_init
    use ocean_module, only: ocean_data
    use grid_module, only: grid_data, grid_global_data
    use io_module, only: read_global_mask
    use init_data_module, only: init_grid_data, init_ocean_data
    use shallow_water_module, only: expl_shallow_water
    use tracer_control_module, only: expl_tracer
    use data_types_module, only: data2D_real8_type, data2D_real4_type
    implicit none

    integer :: nsteps, step, k, ierr, t, ntr
    character(len=256) :: arg, dumpfile
    real(wp8) :: tau
    integer, parameter :: u = 77

    call get_command_argument(1, arg); read(arg, *) nsteps
    call get_command_argument(2, dumpfile)

    call mpp_init()
    call load_config_basinpar_from_file('basin.par')
    call load_config_sw_from_file('sw.par')
    call load_config_parallel_from_file_and_cmd('parallel.par')

    call grid_global_data%init()
    call read_global_mask(grid_global_data)
    call domain_data%init_from_config(grid_global_data%mask)
    call mpp_sync_init(domain_data)
    call ocean_data%init(domain_data)
    call grid_data%init(domain_data)
    call init_grid_data()
    call init_ocean_data()

    tau = 1.0d0
    !$omp parallel default(shared) private(step)
    do step = 1, nsteps
        call expl_shallow_water(tau)
        call expl_tracer(tau)
    enddo
    !$omp end parallel

    if (mpp_rank == 0) then
        open(u, file=trim(dumpfile), access='stream', form='unformatted', status='replace')
        ntr = 0
        if (use_tracers > 0) ntr = tracer_num
        write(u) domain_data%bcount, ntr
        do k = 1, domain_data%bcount
            write(u) domain_data%bindx(k, 1), domain_data%bindx(k, 2),                    &
                     domain_data%bnx_start(k), domain_data%bnx_end(k),                    &
                     domain_data%bny_start(k), domain_data%bny_end(k),                    &
                     domain_data%bbnd_x1(k), domain_data%bbnd_x2(k),                      &
                     domain_data%bbnd_y1(k), domain_data%bbnd_y2(k)
            ! r4 grid fields (order = tests/golden/gen_golden.py R4_FIELDS)
            write(u) grid_data%lu%block(k)%field, grid_data%luu%block(k)%field,           &
                     grid_data%luh%block(k)%field, grid_data%lcu%block(k)%field,          &
                     grid_data%lcv%block(k)%field, grid_data%llu%block(k)%field,          &
                     grid_data%llv%block(k)%field,                                        &
                     grid_data%dx%block(k)%field, grid_data%dy%block(k)%field,            &
                     grid_data%dxt%block(k)%field, grid_data%dyt%block(k)%field,          &
                     grid_data%dxh%block(k)%field, grid_data%dyh%block(k)%field,          &
                     grid_data%dxb%block(k)%field, grid_data%dyb%block(k)%field,          &
                     grid_data%rlh_s%block(k)%field, ocean_data%r_diss%block(k)%field
            ! r8 fields (order = tests/golden/gen_golden.py R8_FIELDS)
            write(u) ocean_data%ssh%block(k)%field, ocean_data%sshn%block(k)%field,       &
                     ocean_data%sshp%block(k)%field,                                      &
                     ocean_data%ubrtr%block(k)%field, ocean_data%ubrtrn%block(k)%field,   &
                     ocean_data%ubrtrp%block(k)%field,                                    &
                     ocean_data%vbrtr%block(k)%field, ocean_data%vbrtrn%block(k)%field,   &
                     ocean_data%vbrtrp%block(k)%field,                                    &
                     grid_data%hhq%block(k)%field, grid_data%hhq_p%block(k)%field,        &
                     grid_data%hhq_n%block(k)%field,                                      &
                     grid_data%hhu%block(k)%field, grid_data%hhu_p%block(k)%field,        &
                     grid_data%hhu_n%block(k)%field,                                      &
                     grid_data%hhv%block(k)%field, grid_data%hhv_p%block(k)%field,        &
                     grid_data%hhv_n%block(k)%field,                                      &
                     grid_data%hhh%block(k)%field, grid_data%hhh_p%block(k)%field,        &
                     grid_data%hhh_n%block(k)%field, grid_data%hhq_rest%block(k)%field,   &
                     ocean_data%vort%block(k)%field, ocean_data%str_t%block(k)%field,     &
                     ocean_data%str_s%block(k)%field, ocean_data%mu%block(k)%field,       &
                     ocean_data%RHSx%block(k)%field, ocean_data%RHSy%block(k)%field,      &
                     ocean_data%RHSx_adv%block(k)%field, ocean_data%RHSy_adv%block(k)%field, &
                     ocean_data%RHSx_dif%block(k)%field, ocean_data%RHSy_dif%block(k)%field
            if (ntr > 0) then
                write(u) ocean_data%flux_x%block(k)%field, ocean_data%flux_y%block(k)%field
                do t = 1, ntr
                    write(u) ocean_data%ff1(t)%block(k)%field, ocean_data%ff1p(t)%block(k)%field,  &
                             ocean_data%ff1n(t)%block(k)%field
                enddo
            endif
        enddo
        close(u)
    endif

    call mpi_finalize(ierr)
end program ref_driver

! ocn_sw_driver.f90 -- Fortran host program: the reference's model.f90 time loop with the
! shallow-water step running on the MI355X through libocn_sw.
!
! usage (in a directory holding basin.par, sw.par, parallel.par):
!     ocn_sw_driver NSTEPS DUMPFILE [native|stages]
! Reads the positional .par files (first lexeme per line, readpar semantics), builds the model
! (decomposition + init_grid_data + init_ocean_data on the device), runs NSTEPS of
! expl_shallow_water + expl_tracer through the Fortran PSy layer -- by default its fused form (one
! ocn_ctx_step per time step), with "stages" the reference's envoke stages, with "native" one
! ocn_ctx_step call of NSTEPS -- and writes every field of every block in the oracle/ref_driver.f90
! dump format.
program ocn_sw_driver
    use iso_c_binding
    use ocn_sw_c
    use ocn_psy
    implicit none

    integer :: nsteps, step, k, id, u, nx, ny, nlo, ntr
    character(len=512) :: arg, dumpfile, maskfile, topofile
    character(len=256) :: lines(32)
    type(ocn_basin) :: basin
    type(ocn_sw_params) :: sw
    type(ocn_decomp) :: dec
    type(ocn_block_info) :: info
    type(c_ptr) :: c
    integer(c_int32_t), allocatable, target :: mask(:, :)
    real(c_float), allocatable, target :: a4(:, :)
    real(c_double), allocatable, target :: a8(:, :)
    real(c_float), allocatable, target :: topo(:, :)
    logical :: native
    integer, parameter :: r4_order(17) = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]

    call get_command_argument(1, arg); read(arg, *) nsteps
    call get_command_argument(2, dumpfile)
    call get_command_argument(3, arg); native = (trim(arg) == 'native')
    if (trim(arg) == 'stages') psy_fused = .false.

    ! basin.par (configs/basinpar.f90:53-77)
    call read_par('basin.par', lines, nlo)
    read(lines(1), *) basin%nx; read(lines(2), *) basin%ny
    read(lines(6), *) basin%dxst; read(lines(7), *) basin%dyst
    read(lines(8), *) basin%rlon; read(lines(9), *) basin%rlat
    read(lines(12), *) basin%curve_grid
    read(lines(13), *) basin%rotation_on_lon; read(lines(14), *) basin%rotation_on_lat
    maskfile = lines(19)
    topofile = lines(20)
    ! sw.par (configs/sw.f90:34-41)
    call read_par('sw.par', lines, nlo)
    read(lines(1), *) sw%full_free_surface; read(lines(2), *) sw%trans_terms; read(lines(3), *) sw%ksw_lat
    read(lines(4), *) sw%time_smooth; read(lines(5), *) sw%lvisc_2
    read(lines(6), *) sw%use_tracers; read(lines(7), *) sw%tracer_num
    ! parallel.par (configs/parallel.f90:34-37), _DD_MANUAL_BLOCK_GRID_
    call read_par('parallel.par', lines, nlo)
    read(lines(3), *) dec%bnx; read(lines(4), *) dec%bny
    dec%nranks = 1; dec%rank = 0; dec%device = 0

    nx = basin%nx; ny = basin%ny
    if (trim(maskfile) == 'none') then
        call ocn_check(ocn_ctx_create(basin, sw, dec, c_null_ptr, c), 'ocn_ctx_create')
    else
        allocate(mask(nx, ny))
        call read_mask(trim(maskfile), nx, ny, mask)
        call ocn_check(ocn_ctx_create(basin, sw, dec, c_loc(mask), c), 'ocn_ctx_create')
    endif
    call psy_init(c, sw)
    if (len_trim(topofile) > 0 .and. trim(topofile) /= 'none') then   ! init_data.f90:115-120
        allocate(topo(nx - 4, ny - 4))
        open(newunit=u, file=trim(topofile), access='stream', form='unformatted', status='old', action='read')
        read(u) topo
        close(u)
        call ocn_check(ocn_ctx_set_topography(c, c_loc(topo), int(size(topo), c_int64_t)), 'set_topography')
    endif
    call ocn_check(ocn_ctx_init_state(c), 'ocn_ctx_init_state')

    if (native) then
        call ocn_check(ocn_ctx_step(c, 1.0d0, int(nsteps, c_int32_t), 1_c_int32_t), 'ocn_ctx_step')
    else
        do step = 1, nsteps                       ! model.f90:146-160
            call expl_shallow_water(1.0d0)
            call expl_tracer(1.0d0)
        enddo
    endif
    call ocn_check(ocn_ctx_synchronize(c), 'ocn_ctx_synchronize')

    open(newunit=u, file=trim(dumpfile), access='stream', form='unformatted', status='replace')
    ntr = 0
    if (sw%use_tracers > 0) ntr = sw%tracer_num
    write(u) int(bcount, c_int32_t), int(ntr, c_int32_t)
    do k = 1, bcount
        call ocn_check(ocn_ctx_block_info(c, int(k - 1, c_int), info), 'block_info')
        write(u) info%bm, info%bn, info%geom%nx_start, info%geom%nx_end, info%geom%ny_start, info%geom%ny_end, &
                 info%geom%bnd_x1, info%geom%bnd_x2, info%geom%bnd_y1, info%geom%bnd_y2
        allocate(a4(info%geom%bnd_x1:info%geom%bnd_x2, info%geom%bnd_y1:info%geom%bnd_y2))
        allocate(a8(info%geom%bnd_x1:info%geom%bnd_x2, info%geom%bnd_y1:info%geom%bnd_y2))
        do id = 1, 17
            call ocn_check(ocn_ctx_download(c, int(k - 1, c_int), int(r4_order(id), c_int), c_loc(a4)), 'download')
            write(u) a4
        enddo
        do id = OCN_SSH, OCN_FIELD_END - 1 + merge(2 + 3 * ntr, 0, ntr > 0)   ! + flux_x, flux_y, ff1/ff1p/ff1n
            call ocn_check(ocn_ctx_download(c, int(k - 1, c_int), int(id, c_int), c_loc(a8)), 'download')
            write(u) a8
        enddo
        deallocate(a4, a8)
    enddo
    close(u)
    call ocn_check(ocn_ctx_destroy(c), 'ocn_ctx_destroy')

contains

    ! legacy/service/read_write_parameters.f90:7-42 semantics: first lexeme of each line
    subroutine read_par(fname, out, n)
        character(*), intent(in) :: fname
        character(len=256), intent(out) :: out(:)
        integer, intent(out) :: n
        character(len=512) :: ln
        integer :: uu, ios, p
        out = ''
        n = 0
        open(newunit=uu, file=fname, status='old', action='read')
        do
            read(uu, '(a)', iostat=ios) ln
            if (ios /= 0) exit
            n = n + 1
            if (n > size(out)) exit
            ln = adjustl(ln)
            p = scan(ln, ' :')
            if (p > 1) then
                out(n) = ln(1:p - 1)
            else
                out(n) = trim(ln)
            endif
            out(n) = replace_d(out(n))
        enddo
        close(uu)
    end subroutine

    function replace_d(s) result(r)          ! Fortran list-directed reads accept 1.0d0 already;
        character(*), intent(in) :: s        ! kept for clarity of the positional format
        character(len=256) :: r
        r = s
    end function

    ! tools/io.f90:61-70: a comment line, then ny rows of nx digits, top row (n = ny) first
    subroutine read_mask(fname, nx, ny, m)
        character(*), intent(in) :: fname
        integer, intent(in) :: nx, ny
        integer(c_int32_t), intent(out) :: m(nx, ny)
        character(len=16) :: frmt
        character(len=80) :: comment
        integer :: uu, i, j
        write(frmt, '(a,i9,a)') '(', nx, 'i1)'
        open(newunit=uu, file=fname, status='old', action='read')
        read(uu, '(a)') comment
        do j = ny, 1, -1
            read(uu, frmt) (m(i, j), i = 1, nx)
        enddo
        close(uu)
    end subroutine

end program ocn_sw_driver

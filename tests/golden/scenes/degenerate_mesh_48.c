#include <stdio.h>
#include <string.h>
#include <stdbool.h>
#include <math.h>
#include <unistd.h>

#include "src/libs/canvas/canvas.h"
#include "src/libs/linalg/linalg.h"
#include "src/libs/obj_loader/obj_loader.h"
#include "src/libs/photon_map/pm.h"
#include "src/color/hsl.h"
#include "src/color/lab.h"
#include "src/color/rgb.h"
#include "src/color/srgb.h"
#include "src/color/xyz.h"
#include "src/color/xyy.h"

#include "src/renderer/camera.h"
#include "src/renderer/config.h"
#include "src/renderer/photon_tracer.h"
#include "src/renderer/renderer.h"
#include "src/renderer/world.h"
#include "src/pattern/pattern.h"
#include "src/shapes/shapes.h"
#include "src/shapes/cone.h"
#include "src/shapes/csg.h"
#include "src/shapes/cube.h"
#include "src/shapes/cylinder.h"
#include "src/shapes/group.h"
#include "src/shapes/plane.h"
#include "src/shapes/sphere.h"
#include "src/shapes/triangle.h"
#include "src/shapes/toroid.h"

#define True true
#define False false

int
main()
{
    /* config */
    struct global_config global_config;
    global_config.illumination.include_direct = True;
    global_config.illumination.include_global = False;
    global_config.illumination.debug_visualize_photon_map = False;
    global_config.illumination.debug_visualize_soft_indirect = False;
    global_config.illumination.di.include_ambient = True;
    global_config.illumination.di.include_diffuse = True;
    global_config.illumination.di.include_specular_highlight = True;
    global_config.illumination.di.include_specular = True;
    global_config.illumination.di.path_length = 5;

    global_config.illumination.gi.include_caustics = True;
    global_config.illumination.gi.include_final_gather = False;
    global_config.illumination.gi.usteps = 8;
    global_config.illumination.gi.vsteps = 8;
    global_config.illumination.gi.irradiance_estimate_num = 200;
    global_config.illumination.gi.irradiance_estimate_radius = 0.1000000000;
    global_config.illumination.gi.irradiance_estimate_cone_filter_k = 1.0000000000;
    global_config.illumination.gi.photon_count = 10000;
    global_config.illumination.gi.path_length = 5;

    global_config.threading.num_threads = 8;
    global_config.scene.divide_threshold = 100000; //1;
    global_config.output.file_path = "/tmp/frt_golden/out/degenerate_mesh_48";
    global_config.output.color_space = SRGB;

    void (*color_space_fn)(const Color, Color) = NULL;
    switch (global_config.output.color_space) {
    case RGB:
        color_space_fn = rgb_to_rgb;
        break;
    case HSL:
        color_space_fn = hsl_to_rgb;
        break;
    case XYZ:
        color_space_fn = xyz_to_rgb;
        break;
    case XYY:
        color_space_fn = xyy_to_rgb;
        break;
    case LAB:
        color_space_fn = lab_to_rgb;
        break;
    case SRGB:
        // this is the default
    default:
        color_space_fn = srgb_to_rgb;
        break;
    }

    /* end config */

    /* camera */
    struct aperture ap;
    aperture(POINT_APERTURE, 0.0, 1, 1, false, &ap);

    Point from = { 0.0000000000, 0.0000000000, -30.0000000000, 1.0 };
    Point to = { 0.0000000000, 0.0000000000, 0.0000000000, 1.0 };
    Vector up = { 0.0000000000, 1.0000000000, 0.0000000000, 0.0 };
    Matrix camera_xform;
    view_transform(from, to, up, camera_xform);

    Camera cam = camera(48, 48, 1.2000000000/*field_of_view*/, 1.0000000000/*distance*/, 1/*usteps*/, 1/*vsteps*/, &ap, camera_xform);

    /* end camera */

    /* lights */
    Light all_lights = array_of_lights(1);

    /* point light 0 */
    Light point_light_0 = all_lights + 0;
    Point point_light_0_point = { -10.0000000000, 10.0000000000, -30.0000000000, 1.0 };
    Color point_light_0_intensity = color(1.0000000000, 1.0000000000, 1.0000000000);
    point_light(point_light_0_point, point_light_0_intensity, point_light_0);

    /* end point light 0 */

    /* end lights */

    /* shapes */
    Shape all_shapes = array_of_shapes(1);

    /* shape 0 */
        Pattern pattern_0_Ka = NULL;
    Pattern pattern_0_Kd = NULL;
    Pattern pattern_0_Ks = NULL;
    Pattern pattern_0_Ns = NULL;
    Pattern pattern_0_bump = NULL;
    Pattern pattern_0_disp = NULL;
    Pattern pattern_0_refl = NULL;
    Pattern pattern_0_d = NULL;
    Color material_0_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_0 = material_alloc();
    color_space_fn(material_0_color_raw, material_0->Ka);
    color_space_fn(material_0_color_raw, material_0->Kd);
    color_space_fn(material_0_color_raw, material_0->Ks);
    color_scale(material_0->Ka, 0.1000000000);
    color_scale(material_0->Kd, 0.8000000000);
    color_scale(material_0->Ks, 0.6000000000);
    rgb_to_rgb(material_0_reflective, material_0->refl);
    rgb_to_rgb(material_0_refractive, material_0->Tf);
    material_0->reflective = material_0_reflective[0] > 0.0
                             || material_0_reflective[1] > 0.0
                             || material_0_reflective[2] > 0.0;

    material_0->Tr = 0.0000000000;
    material_0->Ns = 15.0000000000;
    material_0->Ni = 1.0000000000;
    material_0->casts_shadow = true;
    material_set_pattern(material_0, map_Ka, pattern_0_Ka);
    material_set_pattern(material_0, map_Kd, pattern_0_Kd);
    material_set_pattern(material_0, map_Ks, pattern_0_Ks);
    material_set_pattern(material_0, map_Ns, pattern_0_Ns);
    material_set_pattern(material_0, map_d, pattern_0_d);
    material_set_pattern(material_0, map_bump, pattern_0_bump);
    material_set_pattern(material_0, map_disp, pattern_0_disp);
    material_set_pattern(material_0, map_refl, pattern_0_refl);

    Matrix transform_0, transform_0_tmp;
    matrix_identity(transform_0);
    matrix_rotate_x(-2.2000000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);
    matrix_translate(0.0000000000, -2.0000000000, 0.0000000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);

    Shape shape_0 = all_shapes + 0;

    if (access("scenes/frt_degenerate/degenerate.obj", F_OK ) == -1 ) {
        printf("file 'scenes/frt_degenerate/degenerate.obj' does not exist.");
        return 1;
    }
    printf("Loading resource 'scenes/frt_degenerate/degenerate.obj'... ");
    fflush(stdout);
    construct_group_from_obj_file("scenes/frt_degenerate/degenerate.obj", color_space_fn, shape_0);
    printf("Done!\n");
    fflush(stdout);

    shape_set_material_recursive(shape_0, material_0);
    shape_set_transform(shape_0, transform_0);

    /* end shape 0 */
    /* end shapes */

    Shape world_group = array_of_shapes(1);
    group(world_group, all_shapes, 1);
    printf("Balancing scene...");
    fflush(stdout);
    world_group->divide(world_group, global_config.scene.divide_threshold);
    printf("Done!\n");
    fflush(stdout);

    World w = world();
    w->lights = all_lights;
    w->lights_num = 1;
    w->shapes = world_group;
    w->shapes_num = 1;
    w->global_config = &global_config;

    if (global_config.illumination.gi.photon_count > 0 && (global_config.illumination.include_global  || global_config.illumination.debug_visualize_photon_map || global_config.illumination.debug_visualize_soft_indirect)) {
        w->photon_maps = array_of_photon_maps(3);
        printf("Tracing photons...");
        fflush(stdout);
        int i;
        for (i = 0; i < 3; ++i) {
            init_Photon_map(global_config.illumination.gi.photon_count, w->photon_maps + i);
        }
        trace_photons(w, 3, global_config.illumination.gi.include_caustics, global_config.illumination.gi.include_final_gather);
        printf("Done!\n");
        fflush(stdout);
    } else {
        w->photon_maps = NULL;
        printf("Skipping photon tracing because photon_count is 0.\n");
        fflush(stdout);
    }

    Canvas c = render_multi(cam, w, cam->usteps, cam->vsteps, cam->aperture.jitter);

    write_ppm_file(c, true, global_config.output.file_path);
    write_png(c, global_config.output.file_path);

    canvas_free(c);

    return 0;
}

